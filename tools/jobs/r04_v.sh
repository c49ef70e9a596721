#!/bin/bash
# Round 4, GPU call v: a 128 x 128 conv tile (slot 6): conv parity over every
# listed configuration, then every configuration of the weight-heavy strided /
# ConvT layers in both arithmetics (is tile 6 ever the best?).
set -o pipefail
OUT=gpurun_out/${1:-r04_v}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "config or conv" > "$OUT/pytest_conv.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_conv.log"; step_ok $rc || exit $rc
for prec in f32_ring split16; do
  timeout -k 10 400 python -u tools/layer_bench.py --precision $prec --config all \
      --layers convT2_1024,down2_512,down2_256,convT4_128,dec_in > "$OUT/cfg_$prec.txt" 2>&1 || exit $?
  echo "== $prec"; grep -E "best|tile6 " "$OUT/cfg_$prec.txt" | cut -c1-120
done
