#!/bin/bash
# Round 4, GPU call s: re-time the exact-fp32 headline's launch choices on this
# box (--retune, written to a candidate file) and A/B them against the pinned
# file, interleaved, on the same box.
set -o pipefail
OUT=gpurun_out/${1:-r04_s}
mkdir -p "$OUT"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline --pipeline 1 --no-profile \
    --retune --tuning-out "$OUT/retuned_f32_tuned.json" > "$OUT/retune.json" 2> "$OUT/retune.err" || exit $?
echo "retune run: $(python3 -c "import json;print(json.load(open('$OUT/retune.json'))['ms_per_step'])")"
for r in 1 2 3; do
  for f in profiles/tuning/v2_16x65536_f32_tuned.json "$OUT/retuned_f32_tuned.json"; do
    n=$(basename $f .json)
    timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline --pipeline 1 --no-profile \
        --tuning-in $f > "$OUT/ab_$n.$r.json" 2> "$OUT/ab_$n.$r.err" || exit $?
    echo "$n round $r: $(python3 -c "import json;print(json.load(open('$OUT/ab_$n.$r.json'))['ms_per_step'])")"
  done
done
