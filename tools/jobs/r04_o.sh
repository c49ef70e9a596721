#!/bin/bash
# Round 4, GPU call o: every listed launch configuration of the exact-fp32 ring
# and register-staged convs for the mid-size conv shapes of the v2 step
# (tools/layer_bench.py --config all), to see how far the chosen plan is from
# the best tile for each.
set -o pipefail
OUT=gpurun_out/${1:-r04_o}
mkdir -p "$OUT"
for prec in f32_ring f32; do
  timeout -k 10 400 python -u tools/layer_bench.py --precision $prec --config all \
      --layers convT4_128,down4_64,convT2_1024,down2_256,dec_in,wave > "$OUT/cfg_$prec.txt" 2>&1 || exit $?
  echo "== $prec"; grep -E "best" "$OUT/cfg_$prec.txt"
done
