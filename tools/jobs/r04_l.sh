#!/bin/bash
# Round 4, GPU call l: the fused unit's residual loaded as phase 2 starts
# (variant rp) against the product: unit parity tests on rp, per-unit timings
# in both arithmetics, then the step in both modes, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r04_l}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
RAVE_AMD_LIB_VARIANT=rp timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_range.py tests/test_gpu_parity.py -k "range or residual_unit or fused_units or model_golden" \
    > "$OUT/pytest_rp.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_rp.log"; step_ok $rc || exit $rc
for r in 1 2; do
  for v in "" rp; do
    n=${v:-product}
    for prec in f32_ring split16; do
      RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python -u tools/layer_bench.py --precision $prec \
          --layers unit_64,unit_128,unit_256,unit_512 > "$OUT/units_${n}_$prec.$r.txt" 2>&1 || exit $?
      echo "== $n $prec round $r: $(grep -E '^unit_' $OUT/units_${n}_$prec.$r.txt | awk '{print $1, $3}' | tr '\n' ' ')"
    done
  done
done
for r in 1 2; do
  for v in "" rp; do
    n=${v:-product}
    for prec in f32_tuned auto; do
      RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
          --pipeline 1 --precision $prec > "$OUT/ab_${n}_$prec.$r.json" 2> "$OUT/ab_${n}_$prec.$r.err" || exit $?
      echo "$n $prec round $r: $(python3 -c "import json;d=json.load(open('$OUT/ab_${n}_$prec.$r.json'));print(d['ms_per_step'], {k:round(v['avg_launch_ms']*1e3,2) for k,v in d['roofline']['families'].items()})")"
    done
  done
done
