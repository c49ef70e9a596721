#!/bin/bash
# Fused path edges in both arithmetics: parity, then the default bench line.
set -e -o pipefail
T=${1:-edges}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > $O/pytest_edges.log 2>&1
tail -1 $O/pytest_edges.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cut -c1-300 $O/bench.json
grep -E "head|tail|pqmf|encoder.net.0 |net.21 " $O/bench.err | cut -c1-140
