#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run.  The raw trace is summarised ON THE BOX
# (tools/trace_steps.py) and gzipped so gpurun_out/ stays far below gpurun's 64 MiB merge cap.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench \
  -- python3 bench.py --steps ${STEPS:-4} --warmup ${WARMUP:-3} --no-cpu-baseline --no-parity ${BENCH_ARGS:-} > "$OUT/bench_prof.log" 2>&1
rc=$?
echo "== rocprof rc=$rc"; grep -E '^\{' "$OUT/bench_prof.log" | tail -1
python3 tools/trace_steps.py "$OUT/bench_kernel_trace.csv" --top 60 --step -2 > "$OUT/step_breakdown.txt" 2>&1
head -45 "$OUT/step_breakdown.txt"
gzip -f "$OUT/bench_kernel_trace.csv"
exit $rc
