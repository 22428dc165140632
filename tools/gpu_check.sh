#!/bin/bash
# GPU-box runner: smoke -> pytest -m gpu -> short bench.  Stops at the first fault/abort/timeout
# (exit codes other than 0/1); ordinary test failures (1) continue so one call reports everything.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-10}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
run smoke 600 python __graft_entry__.py smoke
[ "${SKIP_TESTS:-0}" = 1 ] || run pytest_gpu 1200 python -m pytest tests -m gpu -q --maxfail=40 -p no:cacheprovider
[ "${SKIP_BENCH:-0}" = 1 ] || run bench 600 python bench.py --steps "$STEPS" --warmup 3
