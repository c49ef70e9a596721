#!/bin/bash
# Round 6, GPU call p: the row-sliced conv with neighbouring row tiles placed on
# one XCD (xcd_major).  Parity of the skinny-N configurations, then the C3 block
# latency of the pinned plans (r06_o), three times, against r06_o's A/B numbers
# and the variant library without the placement ("xp0"), interleaved.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/${1:-r06_p}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "gemv" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
    for p in f32_bf3 auto; do
        for v in "" xp0; do
            name=${v:-product}
            RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 tools/c3_trace.py run --precision $p --blocks 64 \
                > "$OUT/lat_${p}_${name}_$r.json" 2> "$OUT/lat_${p}_${name}_$r.err" || { tail -5 "$OUT/lat_${p}_${name}_$r.err"; exit 1; }
            echo "$p $name run $r: $(cat $OUT/lat_${p}_${name}_$r.json)"
        done
    done
done
