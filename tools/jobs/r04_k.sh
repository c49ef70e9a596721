#!/bin/bash
# Round 4, GPU call k: per-phase clock stamps of the exact-fp32 ring units
# (diagnostic library: prologue / phase 1 / seam / phase 2 / epilogue per
# workgroup), then the full profiling pass (tools/profile_round.sh).
set -o pipefail
OUT=gpurun_out/${1:-r04_k}
mkdir -p "$OUT"
RAVE_AMD_DIAG_LIB=1 timeout -k 10 200 python -u tools/layer_bench.py --precision f32_ring \
    --layers unit_64,unit_128,unit_512 > "$OUT/stamps_f32.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/stamps_f32.txt" | cut -c1-330
LB_UNIT_COOP=0 RAVE_AMD_DIAG_LIB=1 timeout -k 10 200 python -u tools/layer_bench.py --precision f32_ring \
    --layers unit_256 > "$OUT/stamps_f32_256.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/stamps_f32_256.txt" | cut -c1-330
bash tools/profile_round.sh ${1:-r04_k}
