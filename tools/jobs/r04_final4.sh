#!/bin/bash
# Round 4, final GPU call (last tree of the round): the driver's round-end checks on the final
# tree (full GPU suite, smoke(), the default bench line).  The profiling pass
# (tools/profile_round.sh) runs as its own call.
set -o pipefail
OUT=gpurun_out/${1:-r04_final4}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -4 "$OUT/smoke.log"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/bench.json'))
print('headline', d['precision'], d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'],
      'exact', d['f32_exact']['ms_per_step'], d['f32_exact']['headline_vs_f32_max_abs'],
      'split16', d['split16_auto']['ms_per_step'], 'pipelined', (d.get('pipelined') or {}).get('ms_per_step'),
      'cpu', d['cpu_baseline']['ms_per_step'], 'tuning', d['tuning'])"
