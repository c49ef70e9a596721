#!/bin/bash
# Round 5, GPU call ae: the bf16x3 C = 64 stack in 12 waves (s12: column waves of
# 2, 2, 2, 2, 1, 1 blocks, three waves per SIMD, 168 VGPRs) against 8 waves (product):
# stack parity on the variant, then tools/stack_bench.py interleaved twice.
set -o pipefail
OUT=gpurun_out/${1:-r05_ae}
mkdir -p "$OUT"
RAVE_AMD_LIB_VARIANT=s12 timeout -k 10 300 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "stack" > "$OUT/pytest_stack.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_stack.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" s12; do
        name=${v:-product}
        echo "== $name run $r"
        lib=$v
        xvoff=""
        env $xvoff RAVE_AMD_LIB_VARIANT=$lib timeout -k 10 200 python3 -u tools/stack_bench.py --precision bf16x3 2>&1 \
            | grep -v amdgpu.ids | grep "C=  64" || exit 1
    done
done
