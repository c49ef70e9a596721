#!/bin/bash
# Round 6, GPU call pf: the final tree's profile of the f32_bf3 headline --
# bench line, rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE and MFMA-busy
# passes of the same command (tools/profile_round.sh, bf3 passes only).
set -o pipefail
timeout -k 10 1100 bash tools/profile_round.sh ${1:-r06_pf} bf3
