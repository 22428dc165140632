set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -m gpu -q -rs -p no:cacheprovider --timeout 300 --timeout-method thread -k "model_logits or plain_adamw or matches_single" -s > gpurun_out/pytest_r3b.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "logits max|grad norms worst|passed|failed" gpurun_out/pytest_r3b.log | tail -40
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/diag_glue.py > gpurun_out/diag_glue.log 2>&1; echo "glue rc=$?"; head -70 gpurun_out/diag_glue.log
BENCH_ARGS="--step-roofline 0" bash tools/gpu_prof.sh
