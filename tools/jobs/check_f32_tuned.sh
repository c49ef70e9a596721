#!/bin/bash
# Full GPU suite, then the default bench line (its f32_exact pass now runs
# RAVE_PREC_F32_TUNED: exact fp32 with autotuned launch choices).
set -o pipefail
O=gpurun_out/f32t; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/f32t/bench.json"))
e = d["f32_exact"]
print(d["ms_per_step"], e["ms_per_step"], e["headline_vs_f32_max_abs"], e["roofline"]["frac"], d["pipelined"]["ms_per_step"])
PY
