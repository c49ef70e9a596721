#!/bin/bash
# One profiling pass of bench.py on the GPU box (run through gpurun):
#   1. the plain bench line (with the CPU baseline),
#   2. rocprofv3 --kernel-trace --stats of the same command (per-kernel times),
#   3./4. separate --pmc FETCH_SIZE / WRITE_SIZE passes (HBM traffic; the two
#      counters do not fit one gfx950 pass),
#   5. a --pmc SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass (MFMA utilisation per family),
# then tools/rocprof_summary.py and tools/mfma_util.py.  Every GPU step has its own time limit and the
# script stops at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 10 --warmup 3"
# the first run records the autotuner's choices; the profiled runs reuse them so
# that no plan-build timing launches enter the traces
timeout -k 10 300 python3 $BENCH --tuning-out "$OUT/tuning.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench: $(cat $OUT/bench.json)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 $BENCH --no-cpu-baseline --no-f32 --pipeline 1 --tuning-in "$OUT/tuning.json" > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err"
echo "kernel-trace pass done"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --pipeline 1 --no-f32 \
    --tuning-in "$OUT/tuning.json" > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
echo "fetch pass done"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --pipeline 1 --no-f32 \
    --tuning-in "$OUT/tuning.json" > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
echo "write pass done"
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/mfma" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --pipeline 1 --no-f32 \
    --tuning-in "$OUT/tuning.json" > "$OUT/bench_mfma.json" 2> "$OUT/bench_mfma.err"
echo "mfma pass done"
MF=$(find "$OUT/mfma" -name '*counter_collection.csv' | head -n 1)
python3 "$R/tools/mfma_util.py" "$MF" "$OUT/bench.json" > "$OUT/mfma_util.json"
head -n 1 "$MF" > "$MF.gemm"; grep -E 'conv1d|split_reduce|unit_kernel|unit_split|stack_split|pqmf|encoder_head|decoder_tail' "$MF" >> "$MF.gemm" || true
rm -f "$MF"
KT=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -n 1)
FE=$(find "$OUT/fetch" -name '*counter_collection.csv' | head -n 1)
WR=$(find "$OUT/write" -name '*counter_collection.csv' | head -n 1)
python3 "$R/tools/rocprof_summary.py" --trace "$KT" --fetch "$FE" --write "$WR" \
    --bench "$OUT/bench.json" --out "$OUT/summary.json" --traffic-out "$OUT/traffic.json" \
    --precision auto
find "$OUT/kt" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
# the exact-fp32 mode's own kernel trace (f32_tuned headline run), so the fp32
# line's fractions are reproducible from rocprof too
timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --precision f32_tuned --no-cpu-baseline --pipeline 1 \
    --tuning-out "$OUT/tuning_f32.json" > "$OUT/bench_f32.json" 2> "$OUT/bench_f32.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_f32" -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --precision f32_tuned --no-cpu-baseline --pipeline 1 \
    --tuning-in "$OUT/tuning_f32.json" > "$OUT/bench_f32_kt.json" 2> "$OUT/bench_f32_kt.err"
KT32=$(find "$OUT/kt_f32" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/rocprof_summary.py" --trace "$KT32" --bench "$OUT/bench_f32.json" --out "$OUT/summary_f32.json" \
    --precision f32_tuned > /dev/null
find "$OUT/kt_f32" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_f32.csv" \;
echo "f32 kernel-trace pass done"
# counter CSVs are large; keep the GEMM-family rows only
for f in "$FE" "$WR"; do
    head -n 1 "$f" > "$f.gemm"; grep -E 'conv1d|split_reduce|unit_kernel|unit_split|stack_split|pqmf|encoder_head|decoder_tail' "$f" >> "$f.gemm" || true
    rm -f "$f"
done
ls -la "$OUT"
