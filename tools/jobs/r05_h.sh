#!/bin/bash
# Round 5, GPU call h: weight-ring depth A/B of the bf16x3 units -- the
# cooperative form's ring (RAVE_US_RC 6 product, 10, 14: the phase-2 steps after
# the hand-off ran at ~40 % of the MFMA rate, r05_g) and the one-workgroup
# form's (RAVE_US_R 3 product, 4) -- unit layers alone and the bench step,
# interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_h}
mkdir -p "$OUT"
for r in 1 2; do
    for v in "" rc10 rc14 r4; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 \
            --layers unit_64,unit_128,unit_256,unit_512 > "$OUT/units_${name}_$r.txt" 2>&1 || exit $?
        echo "== $name run $r"; grep -E "^unit" "$OUT/units_${name}_$r.txt"
        LB_UNIT_COOP=0 RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 \
            --layers unit_256 2>&1 | grep -E "^unit"
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
