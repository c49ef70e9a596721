#!/bin/bash
# Round 5, GPU call b: the full GPU suite, the default bench line (stack and
# bf16x3 tail launch choices timed at plan build), then a same-box A/B of the
# bf16x3 conv weight image: product (three bf16 planes, 6 B per weight) vs
# librave_amd_w4.so (the fp32 image, 4 B per weight, split in registers),
# interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_b}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -25 "$OUT/pytest_gpu.log" | grep -E "passed|failed|FAILED|Error" | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python3 bench.py --tuning-out "$OUT/tuning_f32_bf3.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 tools/jobs/bench_brief.py "$OUT/bench.json"
for r in 1 2; do
    for v in "" w4; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 --tuning-in "$OUT/tuning_f32_bf3.json" > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "A/B $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
exit $rc
