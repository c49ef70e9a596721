#!/bin/bash
# Round 5, GPU call f: re-time every launch choice of the f32_bf3 headline plan
# (the cooperative units' hand-off changed: sc1 loads, no acquire) and pin it,
# then the profiling pass of the headline (tools/profile_round.sh ... bf3:
# bench line, rocprofv3 kernel trace, FETCH / WRITE and MFMA-busy passes).
set -o pipefail
OUT=gpurun_out/${1:-r05_f}
mkdir -p "$OUT"
timeout -k 10 600 python3 bench.py --retune --no-f32 --pipeline 1 --no-cpu-baseline \
    --tuning-out "$OUT/tuning_f32_bf3.json" > "$OUT/bench_retune.json" 2> "$OUT/bench_retune.err" || exit $?
python3 tools/jobs/bench_brief.py "$OUT/bench_retune.json" --short
cp "$OUT/tuning_f32_bf3.json" profiles/tuning/v2_16x65536_f32_bf3.json
timeout -k 10 1000 bash tools/profile_round.sh r05_f bf3 > "$OUT/prof.log" 2>&1
rc=$?; tail -3 "$OUT/prof.log"
python3 tools/jobs/bench_brief.py gpurun_out/prof_r05_f/bench.json
exit $rc
