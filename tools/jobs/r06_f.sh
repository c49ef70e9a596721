#!/bin/bash
# Round 6, GPU call f: the product now carries (1) the bf16x3 tail synthesis
# (A/B'd in r06_e), (2) the bf16x3 encoder-head analysis (timed against the
# exact-fp32 head at plan build), (3) the conv epilogue with every K-group
# finishing a share of the rows (RAVE_CONV_KGPAR; variant "kp0" = the round-5
# group-0 epilogue) and (4) the wide cooperative group at C = 256 (coop_rb = 4,
# a tuner candidate: C3's short blocks).  Steps: re-pin the headline plan (one
# new entry: the bf16x3 head), parity, the bench step product vs kp0 interleaved
# twice, then the default bench line re-pinning C3 / C4 / C5 with the new forms.
set -o pipefail
OUT=gpurun_out/${1:-r06_f}
mkdir -p "$OUT/tuning"
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f32 --no-configs --pipeline 1 \
    --save-tuning > "$OUT/pin.json" 2> "$OUT/pin.err" || { tail -5 "$OUT/pin.err"; exit 1; }
cp profiles/tuning/v2_16x65536_f32_bf3.json "$OUT/tuning/"
python3 -c "import json; t=json.load(open('$OUT/tuning/v2_16x65536_f32_bf3.json')); print([r for r in t if r[0].startswith('head')])"
timeout -k 10 500 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_edges.py tests/test_gpu_headline.py tests/test_gpu_streaming.py > "$OUT/pytest_a.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_a.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -rf --timeout 150 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "conv or cooperative or cached_form" > "$OUT/pytest_b.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_b.log"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
    for v in "" kp0; do
        name=${v:-product}
        RAVE_AMD_LIB_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-f32 \
            --no-configs --pipeline 1 > "$OUT/ab_${name}_$r.json" 2> "$OUT/ab_${name}_$r.err" || exit 1
        echo -n "bench $name run $r: "; python3 tools/jobs/bench_brief.py "$OUT/ab_${name}_$r.json" --short
    done
done
rm -f profiles/tuning/c3_*.json profiles/tuning/c4_*.json profiles/tuning/c5_*.json
timeout -k 10 600 python3 -u bench.py --save-tuning > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
cp profiles/tuning/c*_*.json "$OUT/tuning/"
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['frac'])
for p in ('f32_bf3','auto'):
    c=d['configs'][p]; print(p, 'c3', c['c3']['decode'], c['c3']['encode_decode'], c['c3']['launches_per_block'], 'c4', c['c4']['ms_per_shard'], 'c5', c['c5']['ms_per_shard'])"
