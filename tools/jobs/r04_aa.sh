#!/bin/bash
# Round 4, GPU call aa: the cooperative bf16x3 unit (C = 256 / 512 groups handing
# act2(h) rows over inside the launch, three bf16 planes): unit parity, isolated
# C = 256 / 512 unit times, model + streaming parity, then the bench re-tuned
# (--retune) so the plan can pick the new form, launch choices written out.
set -o pipefail
OUT=gpurun_out/${1:-r04_aa}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_range.py tests/test_gpu_coop.py -k "bf16x3 or coop" > "$OUT/pytest_unit.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_unit.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/layer_bench.py --precision bf16x3 --layers unit_256,unit_512 > "$OUT/units_bf16x3.txt" 2>&1 || exit $?
cut -c1-120 "$OUT/units_bf16x3.txt"
timeout -k 10 600 python -u -m pytest -q -s --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_streaming.py -k "f32_bf3" > "$OUT/pytest_model.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_model.log"; grep "\[parity\]" "$OUT/pytest_model.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --retune --no-cpu-baseline --tuning-out "$OUT/tuning_f32_bf3.json" \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
print(d['precision'], d['ms_per_step'], d['value'], d['gemm_launches_by_family'])
for k, v in d['roofline']['families'].items(): print('  ', k, round(v['avg_launch_ms'] * 1e3, 2), 'us', v['frac'])
e = d['f32_exact']; print('f32_exact', e['ms_per_step'], 'max-abs', e['headline_vs_f32_max_abs'])"
