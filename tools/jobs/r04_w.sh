#!/bin/bash
# Round 4, GPU call w: per-op anatomy of the headline (v2, 16 x 65536) encode and
# decode plans with the pinned launch choices, exact fp32 and auto.
set -o pipefail
OUT=gpurun_out/${1:-r04_w}
mkdir -p "$OUT"
for prec in f32_tuned auto; do
  for plan in encode decode; do
    timeout -k 10 300 python3 tools/plan_ops.py --config v2 --plan $plan --batch 16 --precision $prec \
        --tuning-in profiles/tuning/v2_16x65536_$prec.json > "$OUT/${plan}_$prec.json" 2> "$OUT/${plan}_$prec.err" || exit $?
    python3 -c "
import json; d = json.load(open('$OUT/${plan}_$prec.json')); print('$plan $prec', d['ops'], 'ops', d['sum_us'], 'us')
for r in d['rows']: print('   %-60s k%d p%d %7.2f' % (r['label'], r['kind'], r['precision'], r['us']))"
  done
done
