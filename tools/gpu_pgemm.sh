#!/bin/bash
# GPU-box check of the pipelined panel GEMM: its parity tests, the per-shape census (tiled vs
# pgemm, plain variants, cold caches) and the step with the knob on / off.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pgemm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pgemm_tests.log 2>&1
rc=$?; tail -15 gpurun_out/pgemm_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  timeout -k 10 300 python3 tools/gemm_shapes.py tools/gemm_shapes_7m.txt --max-m 32768 --kinds fwd,dgrad --opt pgemm=$m --reps 5 > gpurun_out/shapes_pg$m.log 2>&1 || { echo "shapes rc=$?"; tail -5 gpurun_out/shapes_pg$m.log; exit 1; }
  tail -1 gpurun_out/shapes_pg$m.log
done
STEPS=20 bash tools/sweep_opt.sh pgemm=0 pgemm=1 pgemm=0 pgemm=1
