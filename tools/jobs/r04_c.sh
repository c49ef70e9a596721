#!/bin/bash
# Round 4, GPU call c: skinny-N + seam tests, C3 latency (plain timing and the
# per-kernel anatomy), the timing-only no-convert conv variant against the
# product (the upper bound of producer-side split planes for the convs), and
# the headline bench line under the pinned launch choices.
set -o pipefail
OUT=gpurun_out/${1:-r04_c}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_cc.py -k "gemv or adain_modes or every_config" > "$OUT/pytest_new.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_new.log"; step_ok $rc || exit $rc
timeout -k 10 400 python3 tools/configs_bench.py --only c3 > "$OUT/c3.json" 2> "$OUT/c3.err" || exit $?
grep -E "C3" "$OUT/c3.err"
for r in 1 2; do
  for v in "" nocvt; do
    n=${v:-product}
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
        --pipeline 1 > "$OUT/ab_$n.$r.json" 2> "$OUT/ab_$n.$r.err" || exit $?
    echo "$n round $r: $(python3 -c "import json;d=json.load(open('$OUT/ab_$n.$r.json'));print(d['ms_per_step'], d['roofline']['families']['conv_split16']['avg_launch_ms'])")"
  done
done
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
head -c 600 "$OUT/bench.json"; echo
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/c3kt" -o run -- \
    python3 "$R/tools/c3_trace.py" run > "$R/$OUT/c3_run.json" 2> "$R/$OUT/c3_run.err" || exit $?
KT=$(find "$R/$OUT/c3kt" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/c3_trace.py" summarize "$KT" > "$R/$OUT/c3_ops.json"
rm -f "$KT"
