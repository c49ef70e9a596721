#!/bin/bash
# Round 5, GPU call i: conv XCD row partitions (config pm = 2/4/8: each XCD reads
# 1/pm of the weight).  Parity of every partitioned config against the oracle and
# bitwise against its batch-major twin, then a re-timing of the f32_bf3 plan
# (conv choices with partitions on offer), the per-key conv diff against the
# pinned file, and a same-box A/B of the step: pinned tuning vs the re-timed one.
set -o pipefail
OUT=gpurun_out/${1:-r05_i}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "xcd_row or every_config" > "$OUT/pytest_conv.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_conv.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --retune --no-f32 --pipeline 1 --no-cpu-baseline \
    --tuning-out "$OUT/tuning_f32_bf3.json" > "$OUT/bench_retune.json" 2> "$OUT/bench_retune.err" || exit $?
python3 tools/jobs/bench_brief.py "$OUT/bench_retune.json" --short
python3 tools/jobs/tuning_diff.py profiles/tuning/v2_16x65536_f32_bf3.json "$OUT/tuning_f32_bf3.json"
for r in 1 2; do
    for v in pinned retuned; do
        tin=profiles/tuning/v2_16x65536_f32_bf3.json
        [ $v = retuned ] && tin="$OUT/tuning_f32_bf3.json"
        timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 --tuning-in "$tin" > "$OUT/ab_${v}_$r.json" 2> "$OUT/ab_${v}_$r.err" || exit $?
        echo -n "A/B $v run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${v}_$r.json" --short
    done
done
