#!/bin/bash
# Round 5, GPU call y: configs 3 / 4 / 5 (tools/configs_bench.py) in f32_bf3 and in
# auto on the final tree (packed bf16x3 split, 8-wave C = 64 stack).
set -o pipefail
OUT=gpurun_out/${1:-r05_y}
mkdir -p "$OUT"
for p in f32_bf3 auto; do
    timeout -k 10 500 python3 -u tools/configs_bench.py --precision $p > "$OUT/configs_$p.json" 2> "$OUT/configs_$p.err" || exit $?
    echo "== $p"; cat "$OUT/configs_$p.json" | head -c 3000; echo
done
