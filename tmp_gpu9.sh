set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r9
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -s -k "model_logits" > gpurun_out/r9/pytest_models.log 2>&1
rc=$?; echo "pytest models rc=$rc"; grep -E "grad-norm relative|grad norms worst|passed|failed|Error" gpurun_out/r9/pytest_models.log | tail -30
[ $rc -le 1 ] || exit $rc
B="timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --step-roofline 0"
for o in 0 1 2 4 8 16 32 64 3 7 127 0; do
  $B --opt skip=$o > gpurun_out/r9/b.log 2>&1 || { tail -5 gpurun_out/r9/b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r9/b.log') if l.startswith('{')][-1]); print('skip=$o', d['ms_per_step'])"
done
