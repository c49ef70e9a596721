#!/bin/bash
# A/B of the XCD-major workgroup remap (common.h xcd_major) on the GPU box:
# variants given as arguments ("" = the product library), three alternating
# bench runs each; step time, pipelined time and per-family launch averages.
set -e -o pipefail
O=gpurun_out/xcd_${TAG:-ab}; mkdir -p $O
for i in 1 2 3; do
  for v in "$@"; do
    n=${v:-product}
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 > $O/bench_${n}_$i.json 2> $O/bench_${n}_$i.err
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); f=d['roofline']['families']; print(sys.argv[2], d['ms_per_step'], 'pipelined', d.get('pipelined',{}).get('ms_per_step'), {k: round(v['avg_launch_ms']*1e3,2) for k,v in f.items()})" $O/bench_${n}_$i.json $n
  done
done
