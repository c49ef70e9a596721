#!/bin/bash
# Round 4, profiling pass of the f32_bf3 headline with the pinned (cooperative
# bf16x3) launch choices: the default bench line, then rocprofv3 kernel trace +
# FETCH_SIZE / WRITE_SIZE + MFMA-busy passes (tools/profile_round.sh ... bf3).
set -o pipefail
timeout -k 10 1100 bash tools/profile_round.sh r04_prof bf3 > gpurun_out/r04_prof.log 2>&1
rc=$?; tail -4 gpurun_out/r04_prof.log; exit $rc
