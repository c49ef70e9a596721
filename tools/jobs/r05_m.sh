#!/bin/bash
# Round 5, GPU call m: bf16x3 conv K-step schedule A/B -- the next window's
# conversion interleaved into the MFMA gaps (product: RAVE_CONV_IGLP=1, 4 VALU
# per gap; iglpv6: 6 per gap; iglp2: raw reads grouped first) against the
# round-4 order (iglp0).  bf16x3 conv parity first, then the plan's conv
# layers at their pinned configurations and the bench step.
set -o pipefail
OUT=gpurun_out/${1:-r05_m}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "conv and (bf16x3 or bf3)" > "$OUT/pytest_conv.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_conv.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" iglp0 iglp2 iglpv6; do
        name=${v:-product}
        echo "== $name run $r"
        for lc in down2_512:5 convT2_1024:5 dec_in:5 down4_64:3 convT4_128:15 down2_256:5; do
            l=${lc%%:*}; c=${lc##*:}
            RAVE_AMD_LIB_VARIANT=$v timeout -k 10 120 python3 -u tools/layer_bench.py --precision bf16x3 \
                --layers $l --config $c 2>&1 | grep -E "^[a-z]" || exit 1
        done
    done
done
for r in 1 2; do
    for v in "" iglp0; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit $?
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
