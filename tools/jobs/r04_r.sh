#!/bin/bash
# Round 4, GPU call r: the one-launch RVQ encode with the next layer's codebook
# split prefetched across each group meeting: RVQ / discrete parity, the C4
# encode_codes anatomy, a kernel trace of it (which RVQ kernels ran, how long),
# and the C4 step.
set -o pipefail
OUT=gpurun_out/${1:-r04_r}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests \
    -k "rvq or discrete or codes" > "$OUT/pytest_rvq.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_rvq.log"; step_ok $rc || exit $rc
timeout -k 10 300 python3 tools/plan_ops.py --config discrete --plan encode_codes --batch 8 > "$OUT/c4_encode_codes.json" \
    2> "$OUT/c4_encode_codes.err" || exit $?
python3 -c "
import json; d = json.load(open('$OUT/c4_encode_codes.json')); print('encode_codes', d['ops'], 'ops', d['sum_us'], 'us')
for r in d['rows'][:3]: print('  ', r)"
R=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/kt" -o run -- \
    python3 "$R/tools/plan_ops.py" --config discrete --plan encode_codes --batch 8 --runs 5 > /dev/null 2>&1) || exit $?
S=$(find "$R/$OUT/kt" -name '*kernel_stats.csv' | head -n 1)
grep -i rvq "$S" | cut -c1-200
timeout -k 10 400 python3 tools/configs_bench.py --only c4 > "$OUT/c4.json" 2> "$OUT/c4.err" || exit $?
grep -E "C4" "$OUT/c4.err" | cut -c1-300
