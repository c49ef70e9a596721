#!/bin/bash
# Same-box A/B of committed launch-choice files (profiles/tuning/candidates/):
# the headline step (auto) and the exact-fp32 step (f32_tuned) under each
# candidate, interleaved over ROUNDS rounds; one JSON line per run.
set -e -o pipefail
OUT=gpurun_out/${1:-tuning_ab}
ROUNDS=${2:-3}
mkdir -p "$OUT"
for r in $(seq 1 $ROUNDS); do
  for f in profiles/tuning/candidates/*_auto.json; do
    n=$(basename $f .json)
    timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline --pipeline 1 --no-profile \
        --tuning-in $f > "$OUT/$n.$r.json" 2>> "$OUT/err.log"
    echo "$n round $r: $(python3 -c "import json;print(json.load(open('$OUT/$n.$r.json'))['ms_per_step'])")"
  done
  for f in profiles/tuning/candidates/*_f32_tuned.json; do
    n=$(basename $f .json)
    timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --precision f32_tuned --no-cpu-baseline --pipeline 1 \
        --no-profile --tuning-in $f > "$OUT/$n.$r.json" 2>> "$OUT/err.log"
    echo "$n round $r: $(python3 -c "import json;print(json.load(open('$OUT/$n.$r.json'))['ms_per_step'])")"
  done
done
