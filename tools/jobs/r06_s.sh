#!/bin/bash
# Round 6, GPU call s: the six C = 256 units of the C3 f32_bf3 plan (8 frames) as
# two row-sliced convs each instead of the fused cooperative unit the tuner picked
# from its eager timing.  C3 encode+decode latency, 64 blocks, interleaved 3 times.
set -o pipefail
OUT=gpurun_out/${1:-r06_s}
mkdir -p "$OUT"
for r in 1 2 3; do
    for v in pinned unfused256; do
        if [ $v = pinned ]; then T=profiles/tuning/c3_f32_bf3.json; else T=profiles/tuning/candidates/c3_f32_bf3_$v.json; fi
        timeout -k 10 300 python3 tools/c3_trace.py run --precision f32_bf3 --blocks 64 --tuning $T \
            > "$OUT/lat_${v}_$r.json" 2> "$OUT/lat_${v}_$r.err" || { tail -5 "$OUT/lat_${v}_$r.err"; exit 1; }
        echo "$v run $r: $(cat $OUT/lat_${v}_$r.json)"
    done
done
