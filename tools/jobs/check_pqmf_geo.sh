#!/bin/bash
# PQMF analysis on its own geometry (8 waves x 1 block): PQMF / model parity,
# the full suite, then the bench line.
set -o pipefail
O=gpurun_out/pa; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 > $O/bench_$i.json 2> $O/bench_$i.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); f=d['roofline']['families']; print(d['ms_per_step'], {k: round(v['avg_launch_ms']*1e3,2) for k,v in f.items()})" $O/bench_$i.json
done
