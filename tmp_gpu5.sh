set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -x > gpurun_out/r5/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r5/pytest.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 tools/bench_vproj.py --reps 10 2>&1 | grep -v amdgpu || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5/bench.log 2>&1; echo "bench rc=$?"
python3 - <<'PY'
import json
d=json.loads([l for l in open('gpurun_out/r5/bench.log') if l.startswith('{')][-1])
print('ms/step', d['ms_per_step'], 'value', d['value'], 'frac', d['roofline']['frac'], 'step', {k: d['roofline']['step'][k] for k in ('bound_ms','native_ops_measured_ms','frac_wall')})
for k,v in d['roofline']['step']['families'].items(): print(k, v['launches'], v['measured_ms'], v['frac'])
PY
