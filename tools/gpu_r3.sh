#!/bin/bash
# GPU-box runner (round 3): smoke -> pytest -m gpu -> bench (with roofline.step).  Each GPU step
# under its own time limit; stops at the first fault / abort / timeout (exit codes other than 0/1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-20}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 30 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_SMOKE:-0}" = 1 ] || run smoke 300 python __graft_entry__.py smoke
[ "${SKIP_TESTS:-0}" = 1 ] || run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rs --maxfail=40 -p no:cacheprovider \
    --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
[ "${SKIP_BENCH:-0}" = 1 ] || run bench 600 python bench.py --steps "$STEPS" --warmup 5 ${BENCH_ARGS:-}
