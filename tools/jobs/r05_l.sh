#!/bin/bash
# Round 5, GPU calls l and n: per-workgroup clock stamps of the f32_bf3 plan's conv
# layers at their pinned launch configurations (diagnostic build: 0 start,
# 1 prologue done, 2 first chunk staged, 3 K loop done, 4 epilogue done; call n
# adds wave 0's summed K-loop weight waits and chunk-end waits).
set -o pipefail
OUT=gpurun_out/${1:-r05_l}
mkdir -p "$OUT"
for lc in down2_512:5 convT2_1024:5 dec_in:5 enc_out:625 down4_64:3 convT4_128:15 down2_256:5; do
    l=${lc%%:*}; c=${lc##*:}
    RAVE_AMD_DIAG_LIB=1 timeout -k 10 120 python3 -u tools/layer_bench.py --precision bf16x3 --layers $l \
        --config $c >> "$OUT/conv_stamps.txt" 2>&1 || exit $?
done
grep -v amdgpu.ids "$OUT/conv_stamps.txt"
