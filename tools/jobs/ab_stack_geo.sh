#!/bin/bash
# Residual-stack geometry variants (stack_split.hip RAVE_S64_NB / RAVE_S64_CB):
# parity subset per variant, then the alternating bench A/B.
set -e -o pipefail
O=gpurun_out/sgeo; mkdir -p $O
for v in sc sd; do
  RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "unit or stack or model_golden" --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
TAG=sgeo bash tools/jobs/ab_xcd.sh "" sc sd
