#!/bin/bash
# Round 5, GPU call aa: the bf16x3 C = 64 unit with four 32-column waves per 32-row
# block (w4c1: RAVE_B64_WGN=4, RAVE_B64_CB=1; 8 waves per workgroup, 128 VGPRs,
# 4 waves per SIMD) against two 64-column waves (product: WGN 2, CB 2; 2 waves per
# SIMD): unit parity on the variant, unit layers and the bench step with the C = 64
# stages as units (tools/jobs/tuning_units64.json) and, as 'stacks', the pinned plan.
set -o pipefail
OUT=gpurun_out/${1:-r05_aa}
mkdir -p "$OUT"
RAVE_AMD_LIB_VARIANT=w4c1 timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "residual_unit and bf16x3" > "$OUT/pytest_unit.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_unit.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in stacks "" w4c1; do
        name=${v:-product}
        lib=$v; tin=tools/jobs/tuning_units64.json
        [ "$v" = stacks ] && lib="" && tin=profiles/tuning/v2_16x65536_f32_bf3.json
        echo "== $name run $r"
        RAVE_AMD_LIB_VARIANT=$lib timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 \
            --layers unit_64 2>&1 | grep -E "^unit" || exit 1
        RAVE_AMD_LIB_VARIANT=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 --tuning-in $tin > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
