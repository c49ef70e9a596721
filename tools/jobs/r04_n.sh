#!/bin/bash
# Round 4, GPU call n: exact-fp32 ring units with phase 1 overlapped with the
# window staging (channel chunks; the nochk variant keeps the chunk order
# without the overlap), and stream plans that keep the fp32 ring kernels off
# rows that are not 16-byte pieces: the full GPU suite, C3/C4/C5 in exact fp32,
# per-unit timings and the exact-fp32 step, product against nochk.
set -o pipefail
OUT=gpurun_out/${1:-r04_n}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_gpu.log"; step_ok $rc || exit $rc
timeout -k 10 500 python3 tools/configs_bench.py --precision f32_tuned > "$OUT/configs_f32_tuned.json" \
    2> "$OUT/configs_f32_tuned.err" || exit $?
grep -E "C3|C4|C5" "$OUT/configs_f32_tuned.err" | cut -c1-220
for r in 1 2; do
  for v in "" nochk; do
    n=${v:-product}
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python -u tools/layer_bench.py --precision f32_ring \
        --layers unit_64,unit_128,unit_256,unit_512 > "$OUT/units_$n.$r.txt" 2>&1 || exit $?
    echo "== $n round $r: $(grep -E '^unit_' $OUT/units_$n.$r.txt | awk '{print $1, $3}' | tr '\n' ' ')"
  done
done
for r in 1 2; do
  for v in "" nochk; do
    n=${v:-product}
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
        --pipeline 1 > "$OUT/ab_$n.$r.json" 2> "$OUT/ab_$n.$r.err" || exit $?
    echo "$n round $r: $(python3 -c "import json;d=json.load(open('$OUT/ab_$n.$r.json'));print(d['ms_per_step'], {k:round(v['avg_launch_ms']*1e3,2) for k,v in d['roofline']['families'].items()})")"
  done
done
