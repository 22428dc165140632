#!/bin/bash
# One deterministic eager bench command run four times under rocprofv3 (kernel trace; FETCH_SIZE;
# WRITE_SIZE; MFMA busy -- separate passes as MI355X_MICROARCH.md prescribes), then the per-family
# table of durations, HBM bytes / GB/s and MFMA utilisation (tools/counter_table.py).
#   OUT=gpurun_out/ctr BENCH_ARGS="--model model_a_7m" bash tools/gpu_counters.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/ctr}
rm -rf "$OUT"; mkdir -p "$OUT"
CMD="python3 bench.py --eager --steps 1 --warmup 1 --no-cpu-baseline --no-parity --step-roofline 0 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- $CMD > "$OUT/trace.log" 2>&1 || { echo trace rc=$?; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- $CMD > "$OUT/fetch.log" 2>&1 || { echo fetch rc=$?; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- $CMD > "$OUT/write.log" 2>&1 || { echo write rc=$?; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/mfma" -o run -- $CMD > "$OUT/mfma.log" 2>&1 || { echo mfma rc=$?; exit 1; }
if [ "${STALL:-1}" = 1 ]; then   # where the wave cycles go (MI355X_MICROARCH.md PMC table: disjoint buckets)
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$OUT/stall" -o run -- $CMD > "$OUT/stall.log" 2>&1 || { echo stall rc=$?; tail -5 "$OUT/stall.log"; exit 1; }
fi
python3 tools/counter_table.py "$OUT" --out "$OUT/counters.json" > "$OUT/counters.txt" && cat "$OUT/counters.txt"
find "$OUT" -name "*.csv" -size +1M -exec gzip -f {} \;
