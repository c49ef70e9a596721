#!/bin/bash
# Round 5, GPU call ac: the eight-K-group bf16x3 conv tile (slot 13: 64 x 64, 16
# waves, two-slot ring): every listed bf16x3 conv configuration against the oracle,
# then the plan's conv layers at their pinned configuration against slot 13 with
# one K-split (config 14), interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_ac}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "conv and (bf16x3 or bf3)" > "$OUT/pytest_conv.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_conv.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for lc in down2_512:5 convT2_1024:5 dec_in:5 down4_64:3 down2_256:5 convT4_128:15; do
        l=${lc%%:*}; c=${lc##*:}
        for cfg in $c 14; do
            timeout -k 10 120 python3 -u tools/layer_bench.py --precision bf16x3 --layers $l --config $cfg 2>&1 \
                | grep -E "^[a-z]" || echo "$l config $cfg: not valid here"
        done
    done
done
