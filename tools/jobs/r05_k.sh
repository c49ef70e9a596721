#!/bin/bash
# Round 5, GPU call k: A/B of the unit's residual loads -- issued after phase 1
# (product, RAVE_US_RESPF=1) against issued in the epilogue (respf0) -- unit
# layers alone and the bench step, interleaved three times.
set -o pipefail
OUT=gpurun_out/${1:-r05_k}
mkdir -p "$OUT"
for r in 1 2 3; do
    for v in "" respf0; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 \
            --layers unit_64,unit_128,unit_256,unit_512 > "$OUT/units_${name}_$r.txt" 2>&1 || exit $?
        echo "== $name run $r"; grep -E "^unit" "$OUT/units_${name}_$r.txt"
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
