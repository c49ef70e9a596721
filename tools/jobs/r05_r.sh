#!/bin/bash
# Round 5, GPU call r: re-time the ten standalone convs of the pinned f32_bf3 plan
# after the packed split (tuning file with their keys removed: every other choice
# pinned), diff against the pinned file, then a same-box A/B of the step.
set -o pipefail
OUT=gpurun_out/${1:-r05_r}
mkdir -p "$OUT"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-f32 --pipeline 1 --no-cpu-baseline \
    --tuning-in tools/jobs/tuning_noconv.json --tuning-out "$OUT/tuning_f32_bf3.json" \
    > "$OUT/bench_retime.json" 2> "$OUT/bench_retime.err" || exit $?
python3 tools/jobs/tuning_diff.py profiles/tuning/v2_16x65536_f32_bf3.json "$OUT/tuning_f32_bf3.json"
for r in 1 2; do
    for v in pinned retimed; do
        tin=profiles/tuning/v2_16x65536_f32_bf3.json
        [ $v = retimed ] && tin="$OUT/tuning_f32_bf3.json"
        timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 --tuning-in "$tin" > "$OUT/ab_${v}_$r.json" 2> "$OUT/ab_${v}_$r.err" || exit $?
        echo -n "A/B $v run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${v}_$r.json" --short
    done
done
