#!/bin/bash
# Two SQ counter passes (each within one gfx950 pass budget) over single-layer
# runs of tools/layer_bench.py; CSVs under gpurun_out/pmc_<tag>/.
#   bash tools/jobs/pmc_layer.sh <tag> <layer_bench args...>
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS"
i=1
for P in "$P1" "$P2"; do
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
        python3 $R/tools/layer_bench.py --iters 3 "$@" > "$OUT/p$i.log" 2>&1
    i=$((i+1))
done
python3 $R/tools/pmc_summary.py "$OUT"/p1/*counter_collection.csv "$OUT"/p2/*counter_collection.csv
