#!/bin/bash
# Round 4, GPU call e: the split-f16 range guard's cost, isolated.  Product vs
# the no-guard variant (RAVE_SPLIT_GUARD=0 everywhere) vs the no-guard +
# no-convert variant, interleaved; timing-only variants skip the output checks.
set -o pipefail
OUT=gpurun_out/${1:-r04_e}
mkdir -p "$OUT"
for r in 1 2; do
  for v in "" noguard nocvt; do
    n=${v:-product}
    flag=""; [ -n "$v" ] && flag="--timing-only-variant"
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
        --pipeline 1 $flag > "$OUT/ab_$n.$r.json" 2> "$OUT/ab_$n.$r.err" || exit $?
    echo "$n round $r: $(python3 -c "import json;d=json.load(open('$OUT/ab_$n.$r.json'));print(d['ms_per_step'], {k:round(v['avg_launch_ms']*1e3,2) for k,v in d['roofline']['families'].items()})")"
  done
done
