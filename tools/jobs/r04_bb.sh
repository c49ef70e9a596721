#!/bin/bash
# Round 4, GPU call bb: configs 3 / 4 / 5 (tools/configs_bench.py) in the f32_bf3
# mode (fp32 on every op, exact fp32 MFMA or bf16x3), beside the earlier auto /
# f32_tuned runs (profiles/r04_m, r04_n, r04_final2).
set -o pipefail
OUT=gpurun_out/${1:-r04_bb}
mkdir -p "$OUT"
timeout -k 10 900 python3 tools/configs_bench.py --precision f32_bf3 > "$OUT/configs_f32_bf3.json" \
    2> "$OUT/configs_f32_bf3.err" || exit $?
grep -E "^C[345]|C3 |C4 |C5 " "$OUT/configs_f32_bf3.err" | cut -c1-200
