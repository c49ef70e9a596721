#!/bin/bash
# Cooperative unit parity subset, layer timings, stamps (diag) and the bench line.
set -e -o pipefail
T=${1:-coopx}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "cooperative or unit_range_guard or residual_unit_kernel or fused_units" \
    --timeout 120 --timeout-method thread > $O/pytest_coop.log 2>&1
tail -1 $O/pytest_coop.log
bash tools/jobs/stamps_units.sh $T
