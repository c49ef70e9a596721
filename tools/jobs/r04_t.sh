#!/bin/bash
# Round 4, GPU call t: the encoder head with its ninth analysis block split over
# every wave, and the fp32 head conv on channel pairs: edge / model parity on
# the product, then product against the previous library (variant prev), both
# arithmetic modes, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r04_t}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_range.py -k "edge or head or golden or range" \
    > "$OUT/pytest_edges.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_edges.log"; step_ok $rc || exit $rc
for r in 1 2; do
  for v in "" prev; do
    n=${v:-product}
    for prec in f32_tuned auto; do
      RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
          --pipeline 1 --precision $prec > "$OUT/ab_${n}_$prec.$r.json" 2> "$OUT/ab_${n}_$prec.$r.err" || exit $?
      echo "$n $prec round $r: $(python3 -c "import json;d=json.load(open('$OUT/ab_${n}_$prec.$r.json'));f=d['roofline']['families'];print(d['ms_per_step'], {k:round(v['avg_launch_ms']*1e3,2) for k,v in f.items() if 'head' in k or 'tail' in k})")"
    done
  done
done
