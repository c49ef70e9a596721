#!/bin/bash
# Round 4, GPU call p: per-op anatomy of configs 4 and 5 (tools/plan_ops.py).
set -o pipefail
OUT=gpurun_out/${1:-r04_p}
mkdir -p "$OUT"
for plan in encode_codes decode_codes; do
  timeout -k 10 300 python3 tools/plan_ops.py --config discrete --plan $plan --batch 8 > "$OUT/c4_$plan.json" \
      2> "$OUT/c4_$plan.err" || exit $?
  python3 -c "
import json; d = json.load(open('$OUT/c4_$plan.json')); print('$plan', d['ops'], 'ops', d['sum_us'], 'us')
for r in d['rows'][:8]: print('  ', r)"
done
