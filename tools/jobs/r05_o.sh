#!/bin/bash
# Round 5, GPU call o: the packed bf16x3 split (pairs through v_cvt_pk_bf16_f32,
# shift / mask back to fp32, packed subtracts) and max-form leaky ReLU in the
# split kernels -- full GPU suite, then unit / conv layers and the bench step
# against the previous build (head), interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_o}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" head; do
        name=${v:-product}
        echo "== $name run $r"
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 200 python3 -u tools/layer_bench.py --precision bf16x3 \
            --layers unit_64,unit_128,unit_256,unit_512 2>&1 | grep -E "^unit" || exit 1
        for lc in down2_512:5 convT2_1024:5 dec_in:5 down4_64:3 convT4_128:15 down2_256:5; do
            l=${lc%%:*}; c=${lc##*:}
            RAVE_AMD_LIB_VARIANT=$v timeout -k 10 120 python3 -u tools/layer_bench.py --precision bf16x3 \
                --layers $l --config $c 2>&1 | grep -E "^[a-z]" || exit 1
        done
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
