#!/bin/bash
# Round 4, GPU call z2: bf16x3 convs after the plane-offset fix (Snake alphas and the surplus DMAs past three-plane buffers) (the split kernels with three bf16 operand
# planes): conv parity (every layer case, every listed launch configuration),
# isolated conv times of the step's convs, model + streaming parity in f32_bf3,
# then the default bench line (f32_bf3 autotuned, launch choices written out).
set -o pipefail
OUT=gpurun_out/${1:-r04_z2}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "bf16x3 and (conv or residual_unit or wide_range)" tests/test_gpu_range.py > "$OUT/pytest_bf3.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_bf3.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/layer_bench.py --precision bf16x3 --config all \
    --layers convT2_1024,down2_512,down2_256,convT4_128,dec_in > "$OUT/cfg_bf16x3.txt" 2>&1 || exit $?
grep -E "best" "$OUT/cfg_bf16x3.txt" | cut -c1-120
timeout -k 10 600 python -u -m pytest -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_streaming.py -k "f32_bf3" > "$OUT/pytest_model.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_model.log"; grep "\[parity\]" "$OUT/pytest_model.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --tuning-out "$OUT/tuning_f32_bf3.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
print(d['precision'], d['ms_per_step'], d['value'], d['gemm_launches_by_family'])
for k, v in d['roofline']['families'].items(): print('  ', k, round(v['avg_launch_ms'] * 1e3, 2), 'us', v['frac'])
e = d['f32_exact']; print('f32_exact', e['ms_per_step'], 'max-abs', e['headline_vs_f32_max_abs'])
f = d['split16_auto']; print('split16_auto', f['ms_per_step'], 'max-abs', f['vs_headline_max_abs'])"
