#!/bin/bash
# Round 4, GPU call b: the new skinny-N conv tests, the full -m gpu suite,
# same-box A/B of the tuning candidates, and the anatomy of a C3 streaming
# block (rocprofv3 kernel trace).  Test FAILURES (pytest rc 1) do not stop the
# later steps; any other non-zero status (crash, abort, time limit) does.
set -o pipefail
OUT=gpurun_out/${1:-r04_b}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "gemv" > "$OUT/pytest_gemv.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gemv.log"; step_ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; step_ok $rc || exit $rc
bash tools/jobs/tuning_ab.sh ${1:-r04_b}/tuning_ab 2 || exit $?
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/c3kt" -o run -- \
    python3 "$R/tools/c3_trace.py" run > "$R/$OUT/c3_run.json" 2> "$R/$OUT/c3_run.err" || exit $?
KT=$(find "$R/$OUT/c3kt" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/c3_trace.py" summarize "$KT" > "$R/$OUT/c3_ops.json"
rm -f "$KT"
head -c 1500 "$R/$OUT/c3_ops.json"
