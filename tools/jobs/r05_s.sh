#!/bin/bash
# Round 5, GPU call s: the bf16x3 residual stack against its three units after the
# packed split (tools/stack_bench.py, C = 64 and 128 at the bench shapes), twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_s}
mkdir -p "$OUT"
for r in 1 2; do
    timeout -k 10 200 python3 -u tools/stack_bench.py --precision bf16x3 2>&1 | grep -v amdgpu.ids | tee -a "$OUT/stack.txt" || exit 1
done
