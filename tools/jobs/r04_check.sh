#!/bin/bash
# Round-4 check on the GPU box: the new tests first, a bench that re-tunes and
# pins its launch choices (profiles/tuning/), then the whole -m gpu suite.
# Every GPU step has its own limit; the script stops at the first failure.
set -e -o pipefail
OUT=gpurun_out/${1:-r04_a}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_coop.py tests/test_gpu_parity.py -k "coop or roundtrip or cooperative" > "$OUT/pytest_new.log" 2>&1
echo "new tests passed"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --retune --save-tuning > "$OUT/bench.json" 2> "$OUT/bench.err"
cp profiles/tuning/*.json "$OUT/" 
echo "bench: $(cat $OUT/bench.json | head -c 300)"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
