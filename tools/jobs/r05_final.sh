#!/bin/bash
# Round 5, final GPU call: the tree as committed -- the full GPU suite, smoke()
# and the default bench line (the driver's own commands), outputs kept under
# gpurun_out/<tag>/ for profiles/<tag>/.
set -o pipefail
OUT=gpurun_out/${1:-r05_final}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -q -rf --timeout 150 --timeout-method thread -m gpu tests \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
cat "$OUT/smoke.log" | grep smoke
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 tools/jobs/bench_brief.py "$OUT/bench.json"
