#!/bin/bash
# Round 6, GPU call q: the C = 256 units of the C3 f32_bf3 plan (8 frames) in other
# forms than the tuner picked (bf16x3, groups of 2): the wide group of 4 in bf16x3,
# the exact-fp32 ring unit in groups of 2 and of 4 (4-byte weight image).  C3
# encode+decode latency, 64 blocks, same box, interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r06_q}
mkdir -p "$OUT"
for r in 1 2; do
    for v in pinned wide256 ring256 ringwide256; do
        if [ $v = pinned ]; then T=profiles/tuning/c3_f32_bf3.json; else T=profiles/tuning/candidates/c3_f32_bf3_$v.json; fi
        timeout -k 10 300 python3 tools/c3_trace.py run --precision f32_bf3 --blocks 64 --tuning $T \
            > "$OUT/lat_${v}_$r.json" 2> "$OUT/lat_${v}_$r.err" || { tail -5 "$OUT/lat_${v}_$r.err"; exit 1; }
        echo "$v run $r: $(cat $OUT/lat_${v}_$r.json)"
    done
done
