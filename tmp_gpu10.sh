set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r10
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r10/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r10/pytest.log | tail -10
[ $rc -le 1 ] || exit $rc
B="timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --step-roofline 0"
for o in "" "--opt swg_min_m=32768" "--opt swg_min_m=8192" "" "--opt swg_min_m=32768"; do
  $B $o > gpurun_out/r10/b.log 2>&1 || { tail -5 gpurun_out/r10/b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r10/b.log') if l.startswith('{')][-1]); print('$o', d['ms_per_step'])"
done
