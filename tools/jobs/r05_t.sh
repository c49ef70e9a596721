#!/bin/bash
# Round 5, GPU call t: the bf16x3 C = 64 residual stack in 8 waves with column
# waves of 3, 3, 2, 2 blocks (5 blocks per SIMD; product, RAVE_B64S_WX=4) against
# 10 waves of 2 blocks (wx0, 6 blocks on two of the SIMDs), and the product
# with its 16-byte window loads off (xv0, RAVE_STACK_XV=0): stack parity first,
# then tools/stack_bench.py interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_t}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "stack" > "$OUT/pytest_stack.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_stack.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" xv0 wx0; do
        name=${v:-product}
        echo "== $name run $r"
        lib=$v; [ "$v" = xv0 ] && lib=""
        xvoff=""; [ "$v" = xv0 ] && xvoff="RAVE_STACK_XV=0"
        env $xvoff RAVE_AMD_LIB_VARIANT=$lib timeout -k 10 200 python3 -u tools/stack_bench.py --precision bf16x3 2>&1 \
            | grep -v amdgpu.ids | grep "C=  64" || exit 1
    done
done
