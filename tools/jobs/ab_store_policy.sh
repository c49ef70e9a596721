#!/bin/bash
# Layer-output store policy (common.h RAVE_YAUX): write-through (sc1) variant
# "wt" against plain stores; parity subset first, then the bench A/B.
set -e -o pipefail
O=gpurun_out/wt; mkdir -p $O
RAVE_AMD_LIB_VARIANT=wt timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "conv or unit or stack or model_golden" --timeout 120 --timeout-method thread > $O/pytest_wt.log 2>&1
echo "wt: $(tail -1 $O/pytest_wt.log)"
TAG=wt bash tools/jobs/ab_xcd.sh "" wt
