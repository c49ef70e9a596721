#!/bin/bash
# Round 6, GPU call c: where the cooperative bf16x3 units' time goes -- the
# coop-detail clock stamps (diag library built with -DRAVE_STAMPS
# -DRAVE_STAMPS_COOP: 0 start, 1 window staged, 2 phase 1, 3 published,
# 4 own phase-2 steps, 5 poll done, 6 partner rows staged) of unit_256 and
# unit_512, with the product timings beside them.
set -o pipefail
OUT=gpurun_out/${1:-r06_c}
mkdir -p "$OUT"
timeout -k 10 120 python -u tools/layer_bench.py --precision bf16x3 --layers unit_128,unit_256,unit_512 > "$OUT/layers.txt" 2>&1 || exit 1
grep -v amdgpu.ids "$OUT/layers.txt"
for r in 1 2; do
RAVE_AMD_DIAG_LIB=1 timeout -k 10 120 python -u tools/layer_bench.py --precision bf16x3 --layers unit_256,unit_512 > "$OUT/stamps_$r.txt" 2>&1 || exit 1
grep -v amdgpu.ids "$OUT/stamps_$r.txt"
done
