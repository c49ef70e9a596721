#!/bin/bash
# Round 5, GPU call e: full GPU suite (cooperative hand-off now reads the
# exchange with sc1 loads, no agent acquire, where one workgroup fits per CU),
# then A/B of the bf16x3 units: product vs nosc1 (the acquire kept) vs nowin
# (timing-only: no window loads -- what hiding the prologue loads could buy),
# unit layers alone and the bench step.
set -o pipefail
OUT=gpurun_out/${1:-r05_e}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -25 "$OUT/pytest_gpu.log" | grep -E "passed|failed|FAILED|Error" | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
    for v in "" nosc1 nowin; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 \
            --layers unit_64,unit_128,unit_256,unit_512 > "$OUT/units_${name}_$r.txt" 2>&1 || exit $?
        echo "== $name run $r"; grep -E "^unit" "$OUT/units_${name}_$r.txt"
        extra=""; [ "$v" = nowin ] && extra="--timing-only-variant"
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 $extra > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
exit $rc
