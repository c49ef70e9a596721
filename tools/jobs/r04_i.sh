#!/bin/bash
# Round 4, GPU call i: the full GPU suite on the product library (two-pass
# unit / stack range guard), then concurrency within a step: B = 8 half-steps on
# 2 streams against the B = 16 step, both arithmetics (bench's pipelined leg).
set -o pipefail
OUT=gpurun_out/${1:-r04_i}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; step_ok $rc || exit $rc
for prec in f32_tuned auto; do
  for cfg in "16 1" "16 2" "8 2" "8 3"; do
    set -- $cfg
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline --no-profile \
        --precision $prec --batch $1 --pipeline $2 > "$OUT/pl_${prec}_b$1_p$2.json" 2> "$OUT/pl_${prec}_b$1_p$2.err" || exit $?
    echo "$prec B=$1 streams=$2: $(python3 -c "
import json;d=json.load(open('$OUT/pl_${prec}_b$1_p$2.json'));p=d.get('pipelined') or {}
print('serial', d['ms_per_step'], 'ms;', 'pipelined', p.get('ms_per_step'), 'ms per', $1, 'clips')")"
  done
done
