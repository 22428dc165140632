set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/vp
B="timeout -k 10 120 python3 tools/bench_vproj.py --reps 10"
$B > gpurun_out/vp/base.log 2>&1 || exit 1
cat gpurun_out/vp/base.log | grep -v amdgpu
for d in 1 2 4 8 16 3 6 7 15 31; do
  $B --kinds fused_train --opt vp_dbg=$d 2>&1 | grep -v amdgpu || exit 1
done
timeout -s KILL 60 rocprofv3 -L > gpurun_out/vp/avail.txt 2>&1; echo "list rc=$?"
cd gpurun_out/vp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d p1 -o p1 --output-format csv -- python3 ../../tools/bench_vproj.py --reps 3 --shapes 7m_s0 --kinds fused_train > p1.log 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d p2 -o p2 --output-format csv -- python3 ../../tools/bench_vproj.py --reps 3 --shapes 7m_s0 --kinds fused_train > p2.log 2>&1; echo "pmc2 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d p3 -o p3 --output-format csv -- python3 ../../tools/bench_pgemm.py fwd 32768 768 192 --reps 5 > p3.log 2>&1; echo "pmc3 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d p4 -o p4 --output-format csv -- python3 ../../tools/bench_pgemm.py fwd 32768 768 192 --reps 5 > p4.log 2>&1; echo "pmc4 rc=$?"
find . -name "*counter_collection.csv" | head
