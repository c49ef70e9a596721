#!/bin/bash
# Round 4, GPU call m: configs 3/4/5 on the current tree in both arithmetic modes
# (tools/configs_bench.py), and the smoke entry point.
set -o pipefail
OUT=gpurun_out/${1:-r04_m}
mkdir -p "$OUT"
for prec in auto f32_tuned; do
  timeout -k 10 500 python3 tools/configs_bench.py --precision $prec > "$OUT/configs_$prec.json" 2> "$OUT/configs_$prec.err" || exit $?
  echo "$prec:"; grep -E "C3|C4|C5" "$OUT/configs_$prec.err" | cut -c1-250
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
tail -4 "$OUT/smoke.log"
