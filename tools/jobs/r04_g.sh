#!/bin/bash
# Round 4, GPU call g: the two-pass range guard of the unit / stack kernels
# (variant library g2): range-guard and unit/stack parity tests on it, then
# product vs g2 vs the no-guard variant, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r04_g}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
RAVE_AMD_LIB_VARIANT=g2 timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_range.py tests/test_gpu_parity.py -k "range or residual_unit or stack or fused_units" \
    > "$OUT/pytest_g2.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_g2.log"; step_ok $rc || exit $rc
for r in 1 2; do
  for v in "" g2 noguard; do
    n=${v:-product}
    flag=""; [ "$v" = noguard ] && flag="--timing-only-variant"
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
        --pipeline 1 $flag > "$OUT/ab_$n.$r.json" 2> "$OUT/ab_$n.$r.err" || exit $?
    echo "$n round $r: $(python3 -c "import json;d=json.load(open('$OUT/ab_$n.$r.json'));print(d['ms_per_step'], {k:round(v['avg_launch_ms']*1e3,2) for k,v in d['roofline']['families'].items()})")"
  done
done
