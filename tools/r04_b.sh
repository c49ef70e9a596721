#!/bin/bash
# Round 4, GPU call b: the full -m gpu suite, same-box A/B of the tuning
# candidates, and the anatomy of a C3 streaming block (rocprofv3 kernel trace).
set -e -o pipefail
OUT=gpurun_out/r04_b
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
bash tools/tuning_ab.sh r04_b/tuning_ab 2
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/c3kt" -o run -- \
    python3 "$R/tools/c3_trace.py" run > "$R/$OUT/c3_run.json" 2> "$R/$OUT/c3_run.err"
KT=$(find "$R/$OUT/c3kt" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/c3_trace.py" summarize "$KT" > "$R/$OUT/c3_ops.json"
rm -f "$KT"
head -c 1500 "$R/$OUT/c3_ops.json"
