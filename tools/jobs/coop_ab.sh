#!/bin/bash
# Fused-unit weight-ring depth A/B (variant libraries built from unit_split.hip
# with RAVE_US_RC / RAVE_US_R) and per-phase stamps of the cooperative unit.
set -e -o pipefail
T=${1:-coopab}; O=gpurun_out/$T; mkdir -p $O
for v in "" rc12 rc20 r6; do
  RAVE_AMD_LIB_VARIANT=$v timeout -k 10 120 python -u tools/layer_bench.py --layers unit_128,unit_256,unit_512 > $O/layers_${v:-base}.txt 2>&1
  LB_UNIT_COOP=0 RAVE_AMD_LIB_VARIANT=$v timeout -k 10 120 python -u tools/layer_bench.py --layers unit_256,unit_512 >> $O/layers_${v:-base}.txt 2>&1
  echo "== ${v:-base}"; grep -v amdgpu.ids $O/layers_${v:-base}.txt
done
RAVE_AMD_DIAG_LIB=1 timeout -k 10 120 python -u tools/layer_bench.py --layers unit_256,unit_512 > $O/stamps.txt 2>&1
LB_UNIT_COOP=0 RAVE_AMD_DIAG_LIB=1 timeout -k 10 120 python -u tools/layer_bench.py --layers unit_256,unit_512 >> $O/stamps.txt 2>&1
grep -v amdgpu.ids $O/stamps.txt
