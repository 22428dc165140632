set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/vp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "vproj or model_logits" > gpurun_out/vp/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|grad norms worst" gpurun_out/vp/pytest.log | tail -30
[ $rc -le 1 ] || exit $rc
B="timeout -k 10 120 python3 tools/bench_vproj.py --reps 10"
$B 2>&1 | grep -v amdgpu || exit 1
for d in 1 2; do $B --kinds fused_train --opt vp_dbg=$d 2>&1 | grep -v amdgpu || exit 1; done
cd gpurun_out/vp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d p5 -o p5 --output-format csv -- python3 ../../tools/bench_vproj.py --reps 3 --shapes 7m_s0 --kinds fused_train > p5.log 2>&1; echo "pmc5 rc=$?"
