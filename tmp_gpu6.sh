set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r6/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r6/pytest.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 tools/bench_vproj.py --reps 10 2>&1 | grep -v amdgpu || exit 1
B="timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --step-roofline 0"
for o in "" "--opt se_gemv=0" "--opt sg_prefetch=1" "--opt dw_fuse=0" "--opt se_gemv=0 --opt sg_prefetch=1 --opt dw_fuse=0" ""; do
  $B $o > gpurun_out/r6/b.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/b.log') if l.startswith('{')][-1]); print('$o', d['ms_per_step'])"
done
OUT=gpurun_out/r6/prof BENCH_ARGS="--step-roofline 0" bash tools/gpu_prof.sh > /dev/null 2>&1; echo "prof rc=$?"
