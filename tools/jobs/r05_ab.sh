#!/bin/bash
# Round 5, GPU call ab: the bf16x3 C = 64 unit with eight 32-column waves per row
# block (w8: RAVE_B64_WGN=8, 256 columns, 16 waves, one workgroup per CU) against four
# (product): unit parity on the variant, unit_64 and the bench step with C = 64 units.
set -o pipefail
OUT=gpurun_out/${1:-r05_ab}
mkdir -p "$OUT"
RAVE_AMD_LIB_VARIANT=w8 timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "residual_unit and bf16x3" > "$OUT/pytest_unit.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_unit.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" w8; do
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
