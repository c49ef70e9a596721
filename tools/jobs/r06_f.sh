#!/bin/bash
# Round 6, GPU call f: the product now carries (1) the bf16x3 tail synthesis
# (A/B'd in r06_e), (2) the bf16x3 encoder-head analysis (timed against the
# exact-fp32 head at plan build) and (3) the conv epilogue with every K-group
# finishing a share of the rows (RAVE_CONV_KGPAR; variant "kp0" = the round-5
# group-0 epilogue).  Conv / edge / headline / streaming parity on the product,
# then the bench step, product against kp0, interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r06_f}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_edges.py tests/test_gpu_headline.py tests/test_gpu_streaming.py > "$OUT/pytest_a.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_a.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "conv" > "$OUT/pytest_conv.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_conv.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" kp0; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --no-configs --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit 1
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
