#!/bin/bash
# Round 4, GPU call q: the one-launch RVQ encode (grouped code splits meeting at
# a per-layer counter): RVQ and discrete-model parity, then the C4 anatomy and
# the C4 step against the per-layer launches (RAVE_RVQ_LAYERED=1 would need a
# variant; the anatomy shows the rvq_encode op directly).
set -o pipefail
OUT=gpurun_out/${1:-r04_q}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests \
    -k "rvq or discrete or codes" > "$OUT/pytest_rvq.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_rvq.log"; step_ok $rc || exit $rc
timeout -k 10 300 python3 tools/plan_ops.py --config discrete --plan encode_codes --batch 8 > "$OUT/c4_encode_codes.json" \
    2> "$OUT/c4_encode_codes.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/c4_encode_codes.json')); print('encode_codes', d['ops'], 'ops', d['sum_us'], 'us')
for r in d['rows'][:4]: print('  ', r)"
timeout -k 10 400 python3 tools/configs_bench.py --only c4 > "$OUT/c4.json" 2> "$OUT/c4.err" || exit $?
grep -E "C4" "$OUT/c4.err" | cut -c1-300
