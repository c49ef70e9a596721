#!/bin/bash
# Round 5, GPU call c: C3 (v2 causal streaming, 2048-sample blocks) anatomy in
# f32_bf3 against auto -- configs_bench's C3 latencies, then a rocprofv3 kernel
# trace of 40 eager blocks per precision (tools/c3_trace.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r05_c}
mkdir -p "$OUT"
for p in f32_bf3 auto; do
    timeout -k 10 400 python3 tools/configs_bench.py --precision $p --only c3 > "$OUT/c3_$p.json" 2> "$OUT/c3_$p.err" || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['c3'] if 'c3' in d else d; print(sys.argv[2], {k: (v.get('latency_ms_median'), v.get('latency_ms_p99')) for k, v in c.items() if isinstance(v, dict)})" "$OUT/c3_$p.json" $p
done
cd /tmp && export TMPDIR=/tmp
for p in f32_bf3 auto; do
    C3_PRECISION=$p timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$p" -o run -- \
        python3 $R/tools/c3_trace.py run > "$OUT/c3_trace_$p.log" 2>&1 || exit $?
    KT=$(find "$OUT/kt_$p" -name '*kernel_trace.csv' | head -n 1)
    python3 $R/tools/c3_trace.py summarize "$KT" > "$OUT/c3_ops_$p.json" || exit $?
    rm -f "$KT"
    python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'launches', d['launches_per_block'], 'busy us', round(d['busy_us_per_block'],1), 'span us', round(d['span_us_per_block'],1))
for k in d['kernels'][:14]: print('   %-80s %5.1f x %6.2f us = %6.1f' % (k['kernel'][:80], k['per_block'], k['avg_us'], k['us_per_block']))" "$OUT/c3_ops_$p.json" $p
done
