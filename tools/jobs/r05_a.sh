#!/bin/bash
# Round 5, first GPU call: the full GPU suite (new: the headline plan vs the
# oracle, f32_bf3 on the v3 / AdaIN / C4 / C5 / streaming tests, the bf16x3
# residual stack, bf16x3 cooperative give-ups, concurrent cooperative engines),
# then the default bench line with the stack launches timed at plan build.
set -o pipefail
OUT=gpurun_out/${1:-r05_a}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -25 "$OUT/pytest_gpu.log" | grep -E "passed|failed|FAILED|Error" | tail -25
# test failures (rc 1) still get the bench; anything else (timeout, crash) ends the call
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python3 bench.py --tuning-out "$OUT/tuning_f32_bf3.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
print('headline', d['precision'], d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'],
      'launches', d['gemm_launches_by_family'],
      'exact', d['f32_exact']['ms_per_step'], d['f32_exact']['headline_vs_f32_max_abs'],
      'split16', d['split16_auto']['ms_per_step'], 'pipelined', (d.get('pipelined') or {}).get('ms_per_step'),
      'cpu', d['cpu_baseline'], 'tuning', d['tuning'])
for k, v in d['roofline']['families'].items(): print(k, v['launches'], round(v['avg_launch_ms']*1e3, 2), 'us', v['frac'])"
exit $rc
