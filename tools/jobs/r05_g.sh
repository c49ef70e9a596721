#!/bin/bash
# Round 5, GPU call g: where the cooperative bf16x3 unit's hand-off time goes --
# clock stamps of the -DRAVE_STAMPS_COOP diagnostic library (0 start, 1 window
# staged, 2 phase 1, 3 published, 4 own phase-2 steps, 5 poll done, 6 partner
# rows staged), at the bench sizes of the C = 256 and 512 units.
set -o pipefail
OUT=gpurun_out/${1:-r05_g}
mkdir -p "$OUT"
RAVE_AMD_DIAG_LIB=1 RAVE_AMD_LIB_VARIANT=diagc timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 \
    --layers unit_256,unit_512 > "$OUT/coop_stamps.txt" 2>&1 || exit $?
RAVE_AMD_DIAG_LIB=1 RAVE_AMD_LIB_VARIANT=diagc timeout -k 10 200 python3 -u tools/layer_bench.py --precision split16 \
    --layers unit_512 >> "$OUT/coop_stamps.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/coop_stamps.txt"
