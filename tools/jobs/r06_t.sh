#!/bin/bash
# Round 6, GPU call t: re-tune the f32_bf3 headline plan on the final build (every
# launch choice timed afresh), then the pinned plan against the re-tuned one, same
# box, interleaved three times (20 steps each, no side legs).
set -o pipefail
OUT=gpurun_out/${1:-r06_t}
mkdir -p "$OUT"
Q="--no-cpu-baseline --no-f32 --no-configs --pipeline 1"
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 $Q --retune --tuning-out "$OUT/retuned.json" \
    > "$OUT/retune.json" 2> "$OUT/retune.err" || { tail -5 "$OUT/retune.err"; exit 1; }
for r in 1 2 3; do
    for v in pinned retuned; do
        if [ $v = pinned ]; then TI=profiles/tuning/v2_16x65536_f32_bf3.json; else TI=$OUT/retuned.json; fi
        timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $Q --tuning-in $TI > "$OUT/ab_${v}_$r.json" 2> "$OUT/ab_${v}_$r.err" || exit 1
        echo -n "$v run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${v}_$r.json" --short
    done
done
python3 tools/jobs/tuning_diff.py profiles/tuning/v2_16x65536_f32_bf3.json "$OUT/retuned.json" | head -40
