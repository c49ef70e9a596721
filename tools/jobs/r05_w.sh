#!/bin/bash
# Round 5, GPU call w: the re-pinned f32_bf3 plan (C = 64 stages as bf16x3 stack
# launches, 30 GEMM launches): the headline-plan tests and the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-r05_w}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_headline.py > "$OUT/pytest_headline.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_headline.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 tools/jobs/bench_brief.py "$OUT/bench.json"
