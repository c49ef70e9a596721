#!/bin/bash
# Per-phase clock stamps of the fused units (diag library) and the plain layer timings.
set -e -o pipefail
O=gpurun_out/${1:-stamps}; mkdir -p $O
timeout -k 10 120 python -u tools/layer_bench.py --layers unit_128,unit_256,unit_512 > $O/layers.txt 2>&1
LB_UNIT_COOP=0 timeout -k 10 120 python -u tools/layer_bench.py --layers unit_256 >> $O/layers.txt 2>&1
grep -v amdgpu.ids $O/layers.txt
if [ -f rave_amd/librave_amd_diag.so ]; then
  RAVE_AMD_DIAG_LIB=1 timeout -k 10 120 python -u tools/layer_bench.py --layers unit_64,unit_128,unit_256,unit_512 > $O/stamps.txt 2>&1
  grep -v amdgpu.ids $O/stamps.txt
fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cut -c1-250 $O/bench.json
