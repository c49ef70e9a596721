#!/bin/bash
# Round 4, GPU call y: bf16x3 units at C = 512 (window sized for dilations <= 4):
# unit parity, isolated C = 512 unit times, model + streaming parity in f32_bf3,
# then the default bench line (headline f32_bf3, f32_exact and split16_auto beside
# it), its launch choices written out to be pinned.
set -o pipefail
OUT=gpurun_out/${1:-r04_y}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "residual_unit" > "$OUT/pytest_unit.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_unit.log"; grep "\[bf16x3\]" "$OUT/pytest_unit.log"; step_ok $rc || exit $rc
for prec in f32_ring bf16x3; do
  timeout -k 10 300 python -u tools/layer_bench.py --precision $prec --layers unit_512 > "$OUT/units_$prec.txt" 2>&1 || exit $?
  echo "== $prec"; cut -c1-120 "$OUT/units_$prec.txt"
done
timeout -k 10 600 python -u -m pytest -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_streaming.py -k "f32_bf3" > "$OUT/pytest_model.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_model.log"; grep "\[parity\]" "$OUT/pytest_model.log"; step_ok $rc || exit $rc
timeout -k 10 600 python3 bench.py --tuning-out "$OUT/tuning_f32_bf3.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
print(d['precision'], d['ms_per_step'], d['value'], d['gemm_launches_by_family'])
for k, v in d['roofline']['families'].items(): print('  ', k, round(v['avg_launch_ms'] * 1e3, 2), 'us', v['frac'])
e = d['f32_exact']; print('f32_exact', e['ms_per_step'], 'max-abs', e['headline_vs_f32_max_abs'])
f = d['split16_auto']; print('split16_auto', f['ms_per_step'], 'max-abs', f['vs_headline_max_abs'])
print('cpu', d['cpu_baseline'])"
