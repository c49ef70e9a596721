#!/bin/bash
# Round 4, GPU call cc: bf16x3 unit geometry A/B -- variant exp = two 32-row
# blocks per wave (MI = 2; C = 64 with 4 column waves, BN = 256), which halves the
# B-fragment LDS reads per MFMA: unit parity on the variant, isolated units
# product vs exp, then the f32_bf3 step product vs exp, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r04_cc}
mkdir -p "$OUT"
RAVE_AMD_LIB_VARIANT=exp timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "residual_unit and bf16x3" > "$OUT/pytest_exp.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_exp.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "scripted_export" > "$OUT/pytest_scripted.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_scripted.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "" exp; do
    n=${v:-product}
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python -u tools/layer_bench.py --precision bf16x3 --layers unit_64,unit_128 \
        > "$OUT/units_$n.$r.txt" 2>&1 || exit $?
    echo "$n $r: $(grep -E '^unit' $OUT/units_$n.$r.txt | awk '{print $1, $3, $4}' | tr '\n' ' ')"
  done
done
for r in 1 2; do
  for v in "" exp; do
    n=${v:-product}
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
        --pipeline 1 --no-profile > "$OUT/ab_$n.$r.json" 2> "$OUT/ab_$n.$r.err" || exit $?
    echo "$n step $r: $(python3 -c "import json;print(json.load(open('$OUT/ab_$n.$r.json'))['ms_per_step'])")"
  done
done
