#!/bin/bash
# Round 5, GPU call q: the profiling pass of the f32_bf3 headline after the packed
# bf16x3 split (tools/profile_round.sh ... bf3: bench line, rocprofv3 kernel
# trace, FETCH / WRITE and MFMA-busy passes), on the pinned plan.
set -o pipefail
OUT=gpurun_out/${1:-r05_q}
mkdir -p "$OUT"
timeout -k 10 1000 bash tools/profile_round.sh ${1:-r05_q} bf3 > "$OUT/prof.log" 2>&1
rc=$?; tail -3 "$OUT/prof.log"
python3 tools/jobs/bench_brief.py gpurun_out/prof_${1:-r05_q}/bench.json
exit $rc
