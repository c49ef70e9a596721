#!/bin/bash
# Round 5, GPU call p: upper bound of producer-side bf16x3 planes for the convs --
# timing-only variant nocvt (RAVE_EXP_NOCVT: plane rows copied from the raw
# window, no act / split; wrong results) against the product: conv layers at
# their pinned configurations and the bench step, interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_p}
mkdir -p "$OUT"
for r in 1 2; do
    for v in "" nocvt; do
        name=${v:-product}
        echo "== $name run $r"
        for lc in down2_512:5 convT2_1024:5 dec_in:5 down4_64:3 convT4_128:15 down2_256:5; do
            l=${lc%%:*}; c=${lc##*:}
            RAVE_AMD_LIB_VARIANT=$v timeout -k 10 120 python3 -u tools/layer_bench.py --precision bf16x3 \
                --layers $l --config $c 2>&1 | grep -E "^[a-z]" || exit 1
        done
        extra=""; [ -n "$v" ] && extra="--timing-only-variant"
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 $extra > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
