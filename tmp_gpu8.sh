set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r8
timeout -k 10 120 python3 tools/bench_vproj.py --reps 10 2>&1 | grep -v amdgpu || exit 1
B="timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity --step-roofline 0"
timeout -k 10 300 python3 tools/diag_attn_bias.py > gpurun_out/r8/attn_bias.log 2>&1; echo "diag rc=$?"; grep -v amdgpu gpurun_out/r8/attn_bias.log | tail -30
for o in 0 1 2 4 8 16 32 64 3 7 127 0; do
  $B --opt skip=$o > gpurun_out/r8/b.log 2>&1 || { tail -5 gpurun_out/r8/b.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r8/b.log') if l.startswith('{')][-1]); print('skip=$o', d['ms_per_step'])"
done
