#!/bin/bash
# Round 5, GPU call ad: the bf16x3 C = 128 unit on 32-column tiles (b128w1:
# RAVE_B128_WGN=1; 512 workgroups of 4 waves, two per CU) against 64-column
# tiles (product: 256 workgroups of 8 waves, one per CU): parity on the variant,
# unit_128 and the bench step (pinned plan), interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_ad}
mkdir -p "$OUT"
RAVE_AMD_LIB_VARIANT=b128w1 timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "residual_unit and bf16x3" > "$OUT/pytest_unit.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_unit.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" b128w1; do
        name=${v:-product}
        echo "== $name run $r"
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 \
            --layers unit_128 2>&1 | grep -E "^unit" || exit 1
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
