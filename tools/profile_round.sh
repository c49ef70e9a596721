#!/bin/bash
# One profiling pass of bench.py on the GPU box (run through gpurun), for the
# arithmetic modes the bench line reports -- the headline (f32_bf3: fp32 on every
# op, exact-fp32 MFMA or bf16x3), f32_tuned (exact fp32 MFMA on every op) and the
# mixed line (auto: split-f16 / fp32 per op):
#   1. the plain bench line (with the CPU baseline), then each mode alone,
#   2. rocprofv3 --kernel-trace --stats of the same command (per-kernel times),
#   3./4. separate --pmc FETCH_SIZE / --pmc WRITE_SIZE passes (HBM traffic; the two
#      counters do not fit one gfx950 pass),
#   5. a --pmc SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass (MFMA utilisation per family),
# then tools/rocprof_summary.py and tools/mfma_util.py; steps 2-5 again for f32_tuned
# and for f32_bf3.
# Every run uses the committed launch choices (profiles/tuning/, bench.py's
# default), so no autotune launches enter the traces and every pass runs the
# same plan.  Every GPU step has its own time limit; the script stops at the
# first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
ONLY=${2:-all}      # all | bf3 (the f32_bf3 headline's passes only)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
QUIET="--no-cpu-baseline --pipeline 1 --no-configs"
timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench: $(head -c 400 $OUT/bench.json)"
gemm_rows() {   # counter CSVs are large; keep the GEMM-family rows only
    head -n 1 "$1" > "$1.gemm"
    grep -E 'conv1d|split_reduce|unit_kernel|unit_split|unit_ring|unit_bf3|stack_split|stack_bf3|pqmf|encoder_head|decoder_tail' "$1" >> "$1.gemm" || true
    rm -f "$1"
}
if [ "$ONLY" = all ]; then
timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --precision auto --no-f32 $QUIET \
    > "$OUT/bench_auto.json" 2> "$OUT/bench_auto.err"
# ---------------------------------------------------------------- mixed mode (auto)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --precision auto --no-f32 $QUIET > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err"
echo "kernel-trace pass done"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision auto --no-f32 $QUIET > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.err"
echo "fetch pass done"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision auto --no-f32 $QUIET > "$OUT/bench_write.json" 2> "$OUT/bench_write.err"
echo "write pass done"
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/mfma" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision auto --no-f32 $QUIET > "$OUT/bench_mfma.json" 2> "$OUT/bench_mfma.err"
echo "mfma pass done"
MF=$(find "$OUT/mfma" -name '*counter_collection.csv' | head -n 1)
python3 "$R/tools/mfma_util.py" "$MF" "$OUT/bench_auto.json" > "$OUT/mfma_util.json"
gemm_rows "$MF"
KT=$(find "$OUT/kt" -name '*kernel_trace.csv' | head -n 1)
FE=$(find "$OUT/fetch" -name '*counter_collection.csv' | head -n 1)
WR=$(find "$OUT/write" -name '*counter_collection.csv' | head -n 1)
python3 "$R/tools/rocprof_summary.py" --trace "$KT" --fetch "$FE" --write "$WR" \
    --bench "$OUT/bench_auto.json" --out "$OUT/summary.json" --traffic-out "$OUT/traffic.json" \
    --precision auto > /dev/null
find "$OUT/kt" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
gemm_rows "$FE"
gemm_rows "$WR"
# ---------------------------------------------------------------- headline: exact fp32 (f32_tuned)
timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --precision f32_tuned --no-f32 $QUIET \
    > "$OUT/bench_f32.json" 2> "$OUT/bench_f32.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_f32" -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --precision f32_tuned --no-f32 $QUIET > "$OUT/bench_f32_kt.json" 2> "$OUT/bench_f32_kt.err"
echo "f32 kernel-trace pass done"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_f32" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision f32_tuned --no-f32 $QUIET > "$OUT/bench_f32_fetch.json" 2> "$OUT/bench_f32_fetch.err"
echo "f32 fetch pass done"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_f32" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision f32_tuned --no-f32 $QUIET > "$OUT/bench_f32_write.json" 2> "$OUT/bench_f32_write.err"
echo "f32 write pass done"
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/mfma_f32" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision f32_tuned --no-f32 $QUIET > "$OUT/bench_f32_mfma.json" 2> "$OUT/bench_f32_mfma.err"
echo "f32 mfma pass done"
MF32=$(find "$OUT/mfma_f32" -name '*counter_collection.csv' | head -n 1)
python3 "$R/tools/mfma_util.py" "$MF32" "$OUT/bench_f32.json" > "$OUT/mfma_util_f32.json"
gemm_rows "$MF32"
KT32=$(find "$OUT/kt_f32" -name '*kernel_trace.csv' | head -n 1)
FE32=$(find "$OUT/fetch_f32" -name '*counter_collection.csv' | head -n 1)
WR32=$(find "$OUT/write_f32" -name '*counter_collection.csv' | head -n 1)
python3 "$R/tools/rocprof_summary.py" --trace "$KT32" --fetch "$FE32" --write "$WR32" --bench "$OUT/bench_f32.json" \
    --out "$OUT/summary_f32.json" --traffic-out "$OUT/traffic_f32_tuned.json" --precision f32_tuned > /dev/null
find "$OUT/kt_f32" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_f32.csv" \;
gemm_rows "$FE32"
gemm_rows "$WR32"
fi
# ---------------------------------------------------------------- headline: f32_bf3
timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 3 --precision f32_bf3 --no-f32 $QUIET \
    > "$OUT/bench_bf3.json" 2> "$OUT/bench_bf3.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt_bf3" -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --precision f32_bf3 --no-f32 $QUIET > "$OUT/bench_bf3_kt.json" 2> "$OUT/bench_bf3_kt.err"
echo "bf3 kernel-trace pass done"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch_bf3" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision f32_bf3 --no-f32 $QUIET > "$OUT/bench_bf3_fetch.json" 2> "$OUT/bench_bf3_fetch.err"
echo "bf3 fetch pass done"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write_bf3" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision f32_bf3 --no-f32 $QUIET > "$OUT/bench_bf3_write.json" 2> "$OUT/bench_bf3_write.err"
echo "bf3 write pass done"
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/mfma_bf3" -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-profile --precision f32_bf3 --no-f32 $QUIET > "$OUT/bench_bf3_mfma.json" 2> "$OUT/bench_bf3_mfma.err"
echo "bf3 mfma pass done"
MFB=$(find "$OUT/mfma_bf3" -name '*counter_collection.csv' | head -n 1)
python3 "$R/tools/mfma_util.py" "$MFB" "$OUT/bench_bf3.json" > "$OUT/mfma_util_bf3.json"
gemm_rows "$MFB"
KTB=$(find "$OUT/kt_bf3" -name '*kernel_trace.csv' | head -n 1)
FEB=$(find "$OUT/fetch_bf3" -name '*counter_collection.csv' | head -n 1)
WRB=$(find "$OUT/write_bf3" -name '*counter_collection.csv' | head -n 1)
python3 "$R/tools/rocprof_summary.py" --trace "$KTB" --fetch "$FEB" --write "$WRB" --bench "$OUT/bench_bf3.json" \
    --out "$OUT/summary_bf3.json" --traffic-out "$OUT/traffic_f32_bf3.json" --precision f32_bf3 > /dev/null
find "$OUT/kt_bf3" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_bf3.csv" \;
gemm_rows "$FEB"
gemm_rows "$WRB"
ls -la "$OUT"
