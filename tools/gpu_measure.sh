#!/bin/bash
# GPU-box measurement pass: bench (JSON line) -> rocprofv3 kernel trace/stats of a short bench ->
# two PMC passes (FETCH_SIZE, WRITE_SIZE) -> per-launch HBM traffic of the probed kernels.
# Stops at the first failure.  Outputs under gpurun_out/measure/.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/measure}
rm -rf "$OUT"; mkdir -p "$OUT"
STEPS=${STEPS:-20}
BA=${BENCH_ARGS:-}   # e.g. "--model model_a_14m_tin64 --batch 256"; PMC entries then go under KEYPFX:<probe>
timeout -k 10 600 python3 bench.py --steps "$STEPS" --warmup 5 $BA > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; tail -20 "$OUT/bench.log"; exit 1; }
grep -E '^\{' "$OUT/bench.log" | tail -1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench \
  -- python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --no-parity $BA > "$OUT/prof.log" 2>&1 || { echo "rocprof rc=$?"; tail -20 "$OUT/prof.log"; exit 1; }
grep -E '^\{' "$OUT/prof.log" | tail -1
python3 tools/trace_steps.py "$OUT/prof/bench_kernel_trace.csv" --top 60 --step -2 > "$OUT/step_breakdown.txt" 2>&1
python3 tools/probe_vs_trace.py "$OUT/prof/bench_kernel_trace.csv" "$OUT/prof.log" "$OUT/bench.log" > "$OUT/probe_vs_trace.txt" 2>&1
cat "$OUT/probe_vs_trace.txt"
gzip -f "$OUT/prof/bench_kernel_trace.csv"
if [ "${PMC:-1}" = 1 ]; then
  # FRESH=1: start from an empty table (entries of kernels the step no longer launches are dropped)
  if [ "${FRESH:-0}" = 1 ]; then echo '{}' > "$OUT/pmc_traffic.json"; else cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json" 2>/dev/null || true; fi
  for PR in ${PMC_PROBES:-gemm_panel outlook_bwd sgemm}; do
    ARGS="--eager --steps 2 --warmup 1 --no-cpu-baseline --no-parity --step-roofline 0 --probe $PR $BA"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_$PR" -o run -- python3 bench.py $ARGS > "$OUT/fetch_$PR.log" 2>&1 || { echo "pmc fetch rc=$?"; exit 1; }
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_$PR" -o run -- python3 bench.py $ARGS > "$OUT/write_$PR.log" 2>&1 || { echo "pmc write rc=$?"; exit 1; }
    python3 tools/pmc_traffic.py "$OUT/fetch_$PR" "$OUT/write_$PR" --probe "$PR" --out "$OUT/pmc_traffic.json" \
      ${KEYPFX:+--key "$KEYPFX:$PR"} ${TAG:+--tag "$TAG"}
    find "$OUT/fetch_$PR" "$OUT/write_$PR" -name "*counter_collection.csv" -exec gzip -f {} \;
    find "$OUT/fetch_$PR" "$OUT/write_$PR" -type f ! -name "*.gz" -delete
  done
fi
du -sh "$OUT"
