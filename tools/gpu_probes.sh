#!/bin/bash
# One short eager-probe bench per kernel family: achieved GB/s, fraction of the 8 TB/s peak,
# average launch time, algorithmic bytes per launch, launches (HIP events).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in ${PROBES:-gemm_panel sgemm outlook_fwd outlook_bwd grid_fwd wgrad}; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-parity --probe $p ${BENCH_ARGS:-} > gpurun_out/probe_$p.log 2>&1 || { echo "$p rc=$?"; exit 1; }
  grep "^{" gpurun_out/probe_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$p', r['achieved'], r['frac'], r['avg_launch_ms'], r['algorithmic_bytes_per_launch'], r['launches'])"
done
