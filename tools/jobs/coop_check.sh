#!/bin/bash
# Cooperative fused unit: parity subset, isolated layer timings (cooperative
# vs one workgroup per slab), then the default bench line.
set -e -o pipefail
T=${1:-coop}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "cooperative or unit_range_guard or residual_unit_kernel" \
    --timeout 120 --timeout-method thread > $O/pytest_coop.log 2>&1
tail -1 $O/pytest_coop.log
timeout -k 10 120 python -u tools/layer_bench.py --layers unit_256,unit_512,k3_256,k1_256,k3_512,k1_512 > $O/layers_coop.txt 2>&1
LB_UNIT_COOP=0 timeout -k 10 120 python -u tools/layer_bench.py --layers unit_256,unit_512 > $O/layers_nocoop.txt 2>&1
RAVE_UNIT_XV=0 timeout -k 10 120 python -u tools/layer_bench.py --layers unit_128,unit_256,unit_512 > $O/layers_noxv.txt 2>&1
cat $O/layers_coop.txt $O/layers_nocoop.txt | grep -v amdgpu.ids
echo "== 4-byte window loads"; grep -v amdgpu.ids $O/layers_noxv.txt
timeout -k 10 120 python -u tools/layer_bench.py --precision f32_ring --layers unit_256,unit_512,k3_512,k1_512 > $O/layers_ring.txt 2>&1
LB_UNIT_COOP=0 timeout -k 10 120 python -u tools/layer_bench.py --precision f32_ring --layers unit_256,unit_512 >> $O/layers_ring.txt 2>&1
timeout -k 10 120 python -u tools/layer_bench.py --precision f32 --layers unit_256,unit_512,k3_512,k1_512 >> $O/layers_ring.txt 2>&1
echo "== fp32"; grep -v amdgpu.ids $O/layers_ring.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cut -c1-400 $O/bench.json
if [ -f rave_amd/librave_amd_diag.so ]; then
  RAVE_AMD_DIAG_LIB=1 timeout -k 10 120 python -u tools/layer_bench.py --layers unit_128,unit_256,unit_512 > $O/stamps.txt 2>&1
  LB_UNIT_COOP=0 RAVE_AMD_DIAG_LIB=1 timeout -k 10 120 python -u tools/layer_bench.py --layers unit_256,unit_512 >> $O/stamps.txt 2>&1
  grep -v amdgpu.ids $O/stamps.txt
fi
