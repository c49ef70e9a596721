#!/bin/bash
# 256-column conv tiles (kSplitTiles slots 8-9): every-config parity on the
# product library, then the alternating bench A/B against the previous library.
set -e -o pipefail
O=gpurun_out/wide; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "conv or model_golden or stream" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo "product: $(tail -1 $O/pytest.log)"
TAG=wide bash tools/jobs/ab_xcd.sh "" prev
