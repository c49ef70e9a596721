#!/bin/bash
# Round 5, GPU call j: the bench step as L micro-batches on L HIP streams
# (tools/lanes_probe.py: 16/L clips per lane, one engine instance each, joined
# at the end of the step) against the one-stream step, f32_bf3.
set -o pipefail
OUT=gpurun_out/${1:-r05_j}
mkdir -p "$OUT"
timeout -k 10 900 python3 -u tools/lanes_probe.py --lanes 1,2,4 --rounds 3 \
    --tuning-out "$OUT/lanes_tuning.json" > "$OUT/lanes.txt" 2> "$OUT/lanes.err"
rc=$?; cat "$OUT/lanes.txt"; tail -3 "$OUT/lanes.err"; exit $rc
