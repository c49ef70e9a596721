#!/bin/bash
# Round 4, GPU call x: the bf16x3 fused unit (fp32 on the bf16 matrix cores, exact
# three-way operand split): unit parity (every unit test, bf16x3 against the
# exact-fp32 ring kernel), isolated unit times in both arithmetics, model parity
# in f32_bf3, then the bench step in f32_bf3 with exact fp32 beside it.
set -o pipefail
OUT=gpurun_out/${1:-r04_x}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "residual_unit" > "$OUT/pytest_unit.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_unit.log"; grep "\[bf16x3\]" "$OUT/pytest_unit.log"; step_ok $rc || exit $rc
for prec in f32_ring bf16x3; do
  timeout -k 10 300 python -u tools/layer_bench.py --precision $prec --layers unit_64,unit_128,unit_256 \
      > "$OUT/units_$prec.txt" 2>&1 || exit $?
  echo "== $prec"; cat "$OUT/units_$prec.txt" | cut -c1-120
done
timeout -k 10 500 python -u -m pytest -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "f32_bf3" > "$OUT/pytest_model.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_model.log"; grep "\[parity\]" "$OUT/pytest_model.log"; step_ok $rc || exit $rc
timeout -k 10 500 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --precision f32_bf3 \
    --tuning-out "$OUT/tuning_f32_bf3.json" > "$OUT/bench_bf3.json" 2> "$OUT/bench_bf3.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/bench_bf3.json'))
print('f32_bf3', d['ms_per_step'], d['gemm_launches_by_family'])
for k, v in d['roofline']['families'].items(): print('  ', k, round(v['avg_launch_ms'] * 1e3, 2), 'us', v['frac'])
e = d['f32_exact']; print('f32_tuned', e['ms_per_step'], 'max-abs vs headline', e['headline_vs_f32_max_abs'])"
