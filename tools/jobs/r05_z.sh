#!/bin/bash
# Round 5, GPU call z: C3 (B = 1 causal streaming, f32_bf3) against the units'
# weight-ring depth: product (one-workgroup form R = 3, cooperative RC = 6)
# against rc14 (cooperative RC = 14) and r6 (one-workgroup R = 6), interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_z}
mkdir -p "$OUT"
for r in 1 2; do
    for v in "" rc14 r6; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 -u tools/configs_bench.py --precision f32_bf3 --only c3 \
            > "$OUT/c3_${name}_$r.json" 2> "$OUT/c3_${name}_$r.err" || exit $?
        echo -n "$name run $r: "; python3 -c "
import json,sys; d=json.load(open('$OUT/c3_${name}_$r.json'))['c3']
print('dec p99', d['decode']['latency_ms_p99'], 'enc+dec median', d['encode_decode']['latency_ms_median'], 'p99', d['encode_decode']['latency_ms_p99'])"
    done
done
