#!/bin/bash
# Round 4, GPU call h: (1) the two-pass range guard with its vote after the
# epilogue stores (variant g2): range / unit / stack tests, then product vs g2 vs
# no-guard step A/B; (2) exact-fp32 ring unit geometries (variants fA, fB): the
# f32_ring unit parity cases on each, then per-unit timings (tools/layer_bench.py).
set -o pipefail
OUT=gpurun_out/${1:-r04_h}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
RAVE_AMD_LIB_VARIANT=g2 timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_range.py tests/test_gpu_parity.py -k "range or residual_unit or stack or fused_units" \
    > "$OUT/pytest_g2.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_g2.log"; step_ok $rc || exit $rc
for v in fA fB; do
  RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_gpu_parity.py -k "residual_unit and f32_ring" > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "$v: $(tail -1 $OUT/pytest_$v.log)"; step_ok $rc || exit $rc
done
for r in 1 2; do
  for v in "" fA fB; do
    n=${v:-product}
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python -u tools/layer_bench.py --precision f32_ring \
        --layers unit_64,unit_128,unit_256,unit_512 > "$OUT/units_$n.$r.txt" 2>&1 || exit $?
    echo "== $n round $r"; grep -v amdgpu.ids "$OUT/units_$n.$r.txt" | grep -E "unit_" | cut -c1-160
  done
done
for r in 1 2; do
  for v in "" g2 noguard; do
    n=${v:-product}
    flag=""; [ "$v" = noguard ] && flag="--timing-only-variant"
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
        --pipeline 1 $flag > "$OUT/ab_$n.$r.json" 2> "$OUT/ab_$n.$r.err" || exit $?
    echo "$n round $r: $(python3 -c "import json;d=json.load(open('$OUT/ab_$n.$r.json'));print(d['ms_per_step'], {k:round(v['avg_launch_ms']*1e3,2) for k,v in d['roofline']['families'].items()})")"
  done
done
