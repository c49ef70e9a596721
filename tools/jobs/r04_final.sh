#!/bin/bash
# Round 4, final GPU call: the driver's round-end checks on the final tree --
# the full GPU suite, smoke(), the default bench line -- plus C3 in both modes.
set -o pipefail
OUT=gpurun_out/${1:-r04_final}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_gpu.log"; step_ok $rc || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -3 "$OUT/smoke.log"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
print('headline', d['ms_per_step'], d['value'], d['roofline']['frac'], 'split16', d['split16_auto']['ms_per_step'],
      'pipelined', (d.get('pipelined') or {}).get('ms_per_step'), 'cpu', d['cpu_baseline']['ms_per_step'])"
for prec in auto f32_tuned; do
  timeout -k 10 400 python3 tools/configs_bench.py --only c3 --precision $prec > "$OUT/c3_$prec.json" \
      2> "$OUT/c3_$prec.err" || exit $?
  echo "$prec: $(grep -E 'C3 encode_decode:' $OUT/c3_$prec.err | cut -c1-160)"
done
