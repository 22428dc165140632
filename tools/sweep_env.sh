#!/bin/bash
# Env-knob sweep on the GPU box: `bash tools/sweep_env.sh VAR v1 v2 ...` -> one bench.py run per value.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -k 10 300 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-parity ${BENCH_ARGS:-} > gpurun_out/sweep_one.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/sweep_one.log; exit 1; }
  echo "$var=$v $(grep -E '^\{' gpurun_out/sweep_one.log | tail -1)" | tee -a gpurun_out/sweep.log | python3 -c "import sys,json; l=sys.stdin.read(); o,j=l.split(' ',1); d=json.loads(j); print(o, d['value'], d['ms_per_step'])"
done
