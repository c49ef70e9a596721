#!/bin/bash
# Round 5, GPU call d: where the bf16x3 residual stack's time goes -- stack vs
# its three units in both arithmetics, then per-workgroup clock stamps of the
# stack and of the bf16x3 units (diagnostic -DRAVE_STAMPS library) -- and the C3
# anatomy in f32_bf3 vs auto (tools/jobs/r05_c.sh).
set -o pipefail
OUT=gpurun_out/${1:-r05_d}
mkdir -p "$OUT"
for p in split16 bf16x3; do
    timeout -k 10 200 python3 -u tools/stack_bench.py --precision $p >> "$OUT/stack.txt" 2>&1 || exit $?
    RAVE_AMD_DIAG_LIB=1 timeout -k 10 200 python3 -u tools/stack_bench.py --precision $p --iters 10 >> "$OUT/stack_stamps.txt" 2>&1 || exit $?
done
grep -v amdgpu.ids "$OUT/stack.txt"; grep -v amdgpu.ids "$OUT/stack_stamps.txt"
RAVE_AMD_DIAG_LIB=1 timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 --layers unit_64,unit_128,unit_256,unit_512 \
    > "$OUT/unit_stamps.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/unit_stamps.txt"
bash tools/jobs/r05_c.sh "${1:-r05_d}/c3"
