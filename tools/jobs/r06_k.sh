#!/bin/bash
# Round 6, GPU call k: C3 block latency, same box, interleaved twice: the pinned
# plans of r06_f (no row-sliced convs) against the plans re-tuned with the
# row-sliced skinny-N conv in r06_j, in f32_bf3 and auto (64 blocks, no profiler);
# then a kernel trace of the new f32_bf3 plan (1 ms host sleep between blocks,
# so the trace splits cleanly into blocks).
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06_k}
mkdir -p "$OUT"
for r in 1 2; do
    for p in f32_bf3 auto; do
        for v in old new; do
            if [ $v = old ]; then T=profiles/tuning/c3_$p.json; else T=profiles/tuning/candidates/c3_${p}_rows.json; fi
            timeout -k 10 300 python3 tools/c3_trace.py run --precision $p --blocks 64 --tuning $T \
                > "$OUT/lat_${p}_${v}_$r.json" 2> "$OUT/lat_${p}_${v}_$r.err" || { tail -5 "$OUT/lat_${p}_${v}_$r.err"; exit 1; }
            echo "$p $v run $r: $(cat $OUT/lat_${p}_${v}_$r.json)"
        done
    done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt" -o run -- \
    python3 $R/tools/c3_trace.py run --precision f32_bf3 --tuning $R/profiles/tuning/candidates/c3_f32_bf3_rows.json --sleep-ms 1 \
    > "$OUT/trace_run.json" 2> "$OUT/trace_run.err" || { tail -5 "$OUT/trace_run.err"; exit 1; }
KT=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -n 1)
python3 $R/tools/c3_trace.py analyse "$KT" --gap-us 500 > "$OUT/c3_f32_bf3.json" || exit 1
rm -rf "$OUT/kt"
python3 -c "import json; d=json.load(open('$OUT/c3_f32_bf3.json')); print({k: v for k, v in d.items() if k != 'kernels'})"
