#!/bin/bash
# Same-box A/B of an environment switch on the whole bench step (alternating runs):
#   tools/jobs/ab_env.sh TAG VAR   (VAR=0 vs VAR=1, e.g. RAVE_UNIT_COOP, RAVE_EDGES)
set -e -o pipefail
T=${1:-abenv}; V=${2:-RAVE_UNIT_COOP}; O=gpurun_out/$T; mkdir -p $O
for i in 1 2 3; do
  for v in 1 0; do
    env $V=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --pipeline 1 > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err
    python3 -c "import json;d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]);print('$V=$v', d['ms_per_step'], d['f32_exact']['ms_per_step'], d['gemm_launches_by_family'])"
  done
done
