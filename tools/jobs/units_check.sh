#!/bin/bash
# Unit / stack kernels: parity subset, then the bench line.
set -e -o pipefail
O=gpurun_out/${1:-units}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "stack or unit or cooperative or model_golden or range" \
    --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
timeout -k 10 120 python -u tools/layer_bench.py --layers unit_64,unit_128,unit_256,unit_512 > $O/layers.txt 2>&1
grep -v amdgpu.ids $O/layers.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['f32_exact']['ms_per_step'], d['pipelined']['ms_per_step'])"
