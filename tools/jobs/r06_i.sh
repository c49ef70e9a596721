#!/bin/bash
# Round 6, GPU call i: the C3 kernel trace of the pinned f32_bf3 plan without the
# host sleep between blocks (r06_g slept 2 ms before each block), to see the
# per-kernel durations at the clocks the bench leg runs at.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06_i}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for p in f32_bf3; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$p" -o run -- \
        python3 $R/tools/c3_trace.py run --precision $p > "$OUT/run_$p.json" 2> "$OUT/run_$p.err" || { tail -5 "$OUT/run_$p.err"; exit 1; }
    KT=$(find "$OUT/kt_$p" -name '*kernel_trace.csv' | head -n 1)
    python3 $R/tools/c3_trace.py analyse "$KT" > "$OUT/c3_$p.json" || exit 1
    rm -rf "$OUT/kt_$p"
    cat "$OUT/run_$p.json"; python3 -c "import json; d=json.load(open('$OUT/c3_$p.json')); print({k: v for k, v in d.items() if k != 'kernels'})"
done
