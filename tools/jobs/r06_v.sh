#!/bin/bash
# Round 6, GPU call v: graph-mode streams run the encoder's speaker fill outside the
# graph, once per speaker.  The streaming / coop / operator-seam tests (with the new
# speaker-change test), then C3 latency with and without it (RAVE_STREAM_SPK_ONCE=0),
# pinned plans, both precisions, interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r06_v}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_streaming.py tests/test_gpu_coop.py tests/test_gpu_cc.py > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for p in f32_bf3 auto; do
        for v in 1 0; do
            RAVE_STREAM_SPK_ONCE=$v timeout -k 10 300 python3 tools/c3_trace.py run --precision $p --blocks 64 \
                > "$OUT/lat_${p}_d${v}_$r.json" 2> "$OUT/lat_${p}_d${v}_$r.err" || { tail -5 "$OUT/lat_${p}_d${v}_$r.err"; exit 1; }
            echo "$p spk_once=$v run $r: $(cat $OUT/lat_${p}_d${v}_$r.json)"
        done
    done
done
