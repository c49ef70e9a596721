#!/bin/bash
# fp32 fused unit: two accumulator chains (product) vs one (RAVE_UNIT_DA=0 variant library).
set -e -o pipefail
O=gpurun_out/${1:-uf32}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "residual_unit_kernel or fused_units or model_golden" \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for v in "" noda "" noda; do
  RAVE_AMD_LIB_VARIANT=$v timeout -k 10 120 python -u tools/layer_bench.py --precision f32 --layers unit_64,unit_128,unit_256,unit_512 > $O/l.txt 2>&1
  echo "== ${v:-da}"; grep -v amdgpu.ids $O/l.txt
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['f32_exact']['ms_per_step'])"
