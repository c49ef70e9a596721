#!/bin/bash
# Round 6, GPU call d: cooperative units -- the publish stores' drain moved
# behind the member's own phase-2 steps, the max |h| exchange kept for split16
# only (variant "dr") against the product: cooperative parity on the variant,
# (the TorchScript engine links the product library: its give-up test is left out)
# unit_256 / unit_512 layer timings and the bench step, interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r06_d}
mkdir -p "$OUT"
RAVE_AMD_LIB_VARIANT=dr timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_coop.py tests/test_gpu_parity.py -k "(coop or cooperative or unit or headline) and not torchscript" > "$OUT/pytest_dr.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_dr.log"
[ $rc -eq 0 ] || exit $rc
RAVE_AMD_LIB_VARIANT=dr timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_headline.py tests/test_gpu_range.py > "$OUT/pytest_dr2.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_dr2.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" dr; do
        name=${v:-product}
        echo "== $name run $r"
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 120 python3 -u tools/layer_bench.py --precision bf16x3 \
            --layers unit_256,unit_512 2>&1 | grep -E "^unit" || exit 1
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --no-configs --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit 1
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
