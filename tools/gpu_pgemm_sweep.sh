#!/bin/bash
# Per-shape knob sweep of the pgemm kernel over the 7M small-M census (cold caches).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pgsweep; mkdir -p $O
for cfg in "$@"; do
  opts=""; for o in ${cfg//,/ }; do opts="$opts --opt $o"; done
  timeout -k 10 300 python3 tools/gemm_shapes.py tools/gemm_shapes_7m.txt --max-m 32768 --kinds ${KINDS:-fwd,dgrad} $opts --reps 5 > "$O/$cfg.log" 2>&1 || { echo "$cfg rc=$?"; tail -5 "$O/$cfg.log"; exit 1; }
  echo "$cfg $(tail -1 $O/$cfg.log)"
done
