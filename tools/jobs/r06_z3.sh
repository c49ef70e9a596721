#!/bin/bash
# Round 6, final tree (after the once-per-speaker stream fill): the GPU
# test suite, smoke, and the default bench line (headline + configs leg + CPU baseline).
set -o pipefail
OUT=gpurun_out/${1:-r06_z3}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['frac'])
for p in ('f32_bf3','auto'):
    c=d['configs'][p]; print(p, 'c3', c['c3']['decode'], c['c3']['encode_decode'], c['c3']['launches_per_block'], 'c4', c['c4']['ms_per_shard'], 'c5', c['c5']['ms_per_shard'])
print(json.dumps(d['cpu_baseline'])[:400])"
