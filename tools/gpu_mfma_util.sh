#!/bin/bash
# MFMA utilisation per kernel family of one eager 7M step (rocprofv3 PMC, its own pass):
# SQ_VALU_MFMA_BUSY_CYCLES (MFMA-pipe cycles summed over SIMDs) / (SQ_BUSY_CYCLES x 4 SIMDs).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/mfma; rm -rf $O; mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 bench.py --eager --steps 2 --warmup 1 --no-cpu-baseline --no-parity ${BENCH_ARGS:-} > $O/run.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/run.log; exit 1; }
f=$(find $O/pmc -name "*counter_collection.csv" | head -1)
python3 tools/mfma_util.py "$f" | tee $O/mfma_util.txt
gzip -f "$f"
