#!/bin/bash
# Round 6, GPU call b: the conv ring drain tied to the ring registers (do-while
# chunk loop, ring_keep after the drain), the stack shape check in stack_runs,
# the residency bound and rave_stream_launches: the GPU test suite, smoke, then
# bench.py with the new configs leg (C3 / C4 / C5 in f32_bf3 and auto) pinning
# their launch choices (--save-tuning writes profiles/tuning/c{3,4,5}_*.json).
set -o pipefail
OUT=gpurun_out/${1:-r06_b}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
timeout -k 10 500 python3 -u bench.py --save-tuning > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
mkdir -p "$OUT/tuning" && cp profiles/tuning/c*_*.json "$OUT/tuning/"
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['frac']); print(json.dumps(d['configs'])[:1500]); print(json.dumps(d['cpu_baseline'])[:600])"
