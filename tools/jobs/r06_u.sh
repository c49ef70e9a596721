#!/bin/bash
# Round 6, GPU call u: the encoder's first strided conv of the C3 f32_bf3 plan (net.5,
# k8 s4, 32 output frames) as a row-sliced conv (16 / 8 rows) instead of the tuned
# MFMA tile + separate split-K reduce, and ("allrows") that plus the three K-split
# skinny convs as row-sliced ones.  C3 encode+decode latency, interleaved 3 times.
set -o pipefail
OUT=gpurun_out/${1:-r06_u}
mkdir -p "$OUT"
for r in 1 2 3; do
    for v in pinned rows16net5 rows8net5 allrows; do
        if [ $v = pinned ]; then T=profiles/tuning/c3_f32_bf3.json; else T=profiles/tuning/candidates/c3_f32_bf3_$v.json; fi
        timeout -k 10 300 python3 tools/c3_trace.py run --precision f32_bf3 --blocks 64 --tuning $T \
            > "$OUT/lat_${v}_$r.json" 2> "$OUT/lat_${v}_$r.err" || { tail -5 "$OUT/lat_${v}_$r.err"; exit 1; }
        echo "$v run $r: $(cat $OUT/lat_${v}_$r.json)"
    done
done
