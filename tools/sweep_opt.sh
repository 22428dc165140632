#!/bin/bash
# Knob sweep on the GPU box: one bench.py run per "--opt" setting given as arguments
# (e.g. `bash tools/sweep_opt.sh sg_per_cu=2 sg_per_cu=3`); JSON lines into gpurun_out/sweep.log.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/sweep.log
for o in "$@"; do
  timeout -k 10 300 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-parity --opt "$o" ${BENCH_ARGS:-} > gpurun_out/sweep_one.log 2>&1 || { echo "$o rc=$?"; tail -5 gpurun_out/sweep_one.log; exit 1; }
  echo "$o $(grep -E '^\{' gpurun_out/sweep_one.log | tail -1)" | tee -a gpurun_out/sweep.log | python3 -c "import sys,json; l=sys.stdin.read(); o,j=l.split(' ',1); d=json.loads(j); print(o, d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])"
done
