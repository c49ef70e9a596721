#!/bin/bash
# Round 6, GPU call j: the row-sliced skinny-N conv (tile 14: whole K per workgroup, one
# launch, no split-K combine).  Parity of every gemv configuration, then C3
# re-tuned and traced in
# f32_bf3 and auto (tools/c3_trace.py) against the r06_g trace of the pinned plans.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06_j}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "gemv or every_config or cached_form" tests/test_gpu_streaming.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for p in f32_bf3 auto; do
    timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$p" -o run -- \
        python3 $R/tools/c3_trace.py run --precision $p --retune --save "$OUT/c3_$p.tuning.json" \
        > "$OUT/run_$p.json" 2> "$OUT/run_$p.err" || { tail -5 "$OUT/run_$p.err"; exit 1; }
    KT=$(find "$OUT/kt_$p" -name '*kernel_trace.csv' | head -n 1)
    python3 $R/tools/c3_trace.py analyse "$KT" > "$OUT/c3_$p.json" || exit 1
    rm -rf "$OUT/kt_$p"
    cat "$OUT/run_$p.json"; python3 -c "import json; d=json.load(open('$OUT/c3_$p.json')); print({k: v for k, v in d.items() if k != 'kernels'})"
done
