#!/bin/bash
# Where the panel GEMM's time goes: the same shapes with parts of its memory traffic switched off
# (knob pg_dbg; results are wrong by design, timing only).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
B="timeout -k 10 120 python3 tools/bench_pgemm.py"
for sh in "fwd 32768 768 192" "fwd 32768 192 768 --act gelu" "dgrad 32768 768 192 --act gelu" "fwd 8192 1024 256" "dgrad 8192 256 1024"; do
  for d in 0 1 2 4 3 7; do
    $B $sh --opt pg_dbg=$d 2>&1 | grep -v amdgpu.ids || exit 1
  done
  $B $sh --opt pg_dbg=0 --opt split_w=0 2>&1 | grep -v amdgpu.ids || exit 1
done
