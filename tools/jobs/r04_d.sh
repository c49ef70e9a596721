#!/bin/bash
# Round 4, GPU call d: cached fused units in the stream plans (parity tests,
# C3 latency with and without them, the per-kernel anatomy), then the
# timing-only no-convert conv variant (split planes made by a raw bit copy: the
# upper bound of producer-side split planes) against the product, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r04_d}
mkdir -p "$OUT"
step_ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_streaming.py tests/test_gpu_speaker.py -k "cached_form or stream" \
    > "$OUT/pytest_stream.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_stream.log"; step_ok $rc || exit $rc
for v in 1 0; do
  RAVE_STREAM_UNITS=$v timeout -k 10 400 python3 tools/configs_bench.py --only c3 > "$OUT/c3_units$v.json" \
      2> "$OUT/c3_units$v.err" || exit $?
  echo "units=$v: $(grep -E "C3" "$OUT/c3_units$v.err" | tail -1)"
done
R=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/$OUT/c3kt" -o run -- \
    python3 "$R/tools/c3_trace.py" run > "$R/$OUT/c3_run.json" 2> "$R/$OUT/c3_run.err") || exit $?
KT=$(find "$R/$OUT/c3kt" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/c3_trace.py" summarize "$KT" > "$R/$OUT/c3_ops.json"
rm -f "$KT"
head -c 300 "$OUT/c3_ops.json"; echo
for r in 1 2; do
  for v in "" nocvt; do
    n=${v:-product}
    flag=""; [ -n "$v" ] && flag="--timing-only-variant"
    RAVE_AMD_LIB_VARIANT=$v timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-f32 --no-cpu-baseline \
        --pipeline 1 $flag > "$OUT/ab_$n.$r.json" 2> "$OUT/ab_$n.$r.err" || exit $?
    echo "$n round $r: $(python3 -c "import json;d=json.load(open('$OUT/ab_$n.$r.json'));print(d['ms_per_step'], d['roofline']['families']['conv_split16']['avg_launch_ms'])")"
  done
done
