#!/bin/bash
# Round 6, GPU call e: the decoder tail's PQMF synthesis in bf16x3 (variant
# "ts": three bf16 planes of the filter and of the synthesis input, six
# v_mfma_f32_16x16x32_bf16 per 32-deep K-step) against the product (exact-fp32
# synthesis): the edge and model parity tests on the variant, then the bench
# step interleaved twice (the tail family's event time rides in the line).
set -o pipefail
OUT=gpurun_out/${1:-r06_e}
mkdir -p "$OUT"
RAVE_AMD_LIB_VARIANT=ts timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_edges.py tests/test_gpu_headline.py > "$OUT/pytest_ts.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_ts.log"
[ $rc -eq 0 ] || exit $rc
RAVE_AMD_LIB_VARIANT=ts timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "golden and f32_bf3" > "$OUT/pytest_ts2.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_ts2.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" ts; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --no-configs --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit 1
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
