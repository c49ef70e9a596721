#!/bin/bash
# Round 5, GPU call v: the pinned f32_bf3 plan (units everywhere) against the same
# plan with the two C = 64 residual stacks taken as bf16x3 stack launches
# (tools/jobs/tuning_stack64.json: 34 -> 30 GEMM launches), interleaved three times.
set -o pipefail
OUT=gpurun_out/${1:-r05_v}
mkdir -p "$OUT"
for r in 1 2 3; do
    for v in pinned stack64; do
        tin=profiles/tuning/v2_16x65536_f32_bf3.json
        [ $v = stack64 ] && tin=tools/jobs/tuning_stack64.json
        timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 --tuning-in "$tin" > "$OUT/ab_${v}_$r.json" 2> "$OUT/ab_${v}_$r.err" || exit $?
        echo -n "A/B $v run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${v}_$r.json" --short
    done
done
