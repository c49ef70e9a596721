#!/bin/bash
# Round 6, GPU call a: the starting point -- bench line (f32_bf3 headline) and the
# per-op event times of the pinned f32_bf3 encode and decode plans.
set -o pipefail
OUT=gpurun_out/${1:-r06_a}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
tail -c 600 "$OUT/bench.json"
for p in encode decode; do
    timeout -k 10 200 python3 -u tools/plan_ops.py --config v2 --plan $p --batch 16 --samples 65536 \
        --precision f32_bf3 --tuning-in profiles/tuning/v2_16x65536_f32_bf3.json > "$OUT/ops_$p.json" 2> "$OUT/ops_$p.err" || exit 1
done
echo done
