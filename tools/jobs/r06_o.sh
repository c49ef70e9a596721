#!/bin/bash
# Round 6, GPU call o: the row-sliced skinny-N conv with its first weight batch in flight
# while the window is staged, later batches loaded under the previous FMAs.  Same steps as
# r06_l: parity, C3 re-tuned and saved as candidates, C3 latency of the r06_f pins against
# them (same box, interleaved twice), and a kernel trace of the new f32_bf3 plan.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06_o}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "gemv or every_config or cached_form" tests/test_gpu_streaming.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for p in f32_bf3 auto; do
    timeout -k 10 300 python3 tools/c3_trace.py run --precision $p --retune --save "$OUT/c3_${p}_rows.json" \
        > "$OUT/tune_$p.json" 2> "$OUT/tune_$p.err" || { tail -5 "$OUT/tune_$p.err"; exit 1; }
done
for r in 1 2; do
    for p in f32_bf3 auto; do
        for v in old new; do
            if [ $v = old ]; then T=profiles/tuning/c3_$p.json; else T=$OUT/c3_${p}_rows.json; fi
            timeout -k 10 300 python3 tools/c3_trace.py run --precision $p --blocks 64 --tuning $T \
                > "$OUT/lat_${p}_${v}_$r.json" 2> "$OUT/lat_${p}_${v}_$r.err" || { tail -5 "$OUT/lat_${p}_${v}_$r.err"; exit 1; }
            echo "$p $v run $r: $(cat $OUT/lat_${p}_${v}_$r.json)"
        done
    done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
    python3 $R/tools/c3_trace.py run --precision f32_bf3 --tuning $OUT/c3_f32_bf3_rows.json --sleep-ms 1 \
    > "$OUT/trace_run.json" 2> "$OUT/trace_run.err" || { tail -5 "$OUT/trace_run.err"; exit 1; }
KT=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -n 1)
python3 $R/tools/c3_trace.py analyse "$KT" --gap-us 500 > "$OUT/c3_f32_bf3.json" || exit 1
rm -rf "$OUT/kt"
python3 -c "import json; d=json.load(open('$OUT/c3_f32_bf3.json')); print({k: v for k, v in d.items() if k != 'kernels'})"
