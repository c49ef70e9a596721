#!/bin/bash
# A/B of kernel variants on the GPU box (run through gpurun):
#   bash tools/jobs/ab.sh <tag> <variant>...   ("" = the product librave_amd.so)
# Per variant: the fixed-cost probe and a short bench (no CPU baseline, no
# exact-fp32 pass); each GPU step has its own time limit, stop at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
OUT=$R/gpurun_out/ab_$TAG
mkdir -p "$OUT"
for v in "$@"; do
    name=${v:-product}
    echo "== $name"
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python3 -u $R/tools/fixed_cost_probe.py > "$OUT/fixed_$name.txt" 2>&1
    grep -E "fit|K=" "$OUT/fixed_$name.txt"
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 -u $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
        > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('bench', d['ms_per_step'], 'ms/step; conv frac', r['families']['conv_split16']['frac'], 'avg us', round(r['families']['conv_split16']['avg_launch_ms']*1e3,2))" "$OUT/bench_$name.json"
done
