#!/bin/bash
# Per-shape timing + SQ counters of the pgemm kernel (tuning).  Outputs under gpurun_out/pgprobe.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/pgprobe; mkdir -p $O
B="timeout -k 10 120 python3 tools/bench_pgemm.py"
for sh in "fwd 32768 768 192" "fwd 32768 192 768 --act gelu" "dgrad 32768 192 768" "dgrad 32768 768 192 --act gelu" "fwd 8192 1024 256" "fwd 8192 256 1024 --act gelu"; do
  for o in "pgemm=1" "pgemm=1 --opt split_w=0" "pgemm=0"; do
    $B $sh --opt $o >> $O/times.log 2>&1 || { echo fail; tail -3 $O/times.log; exit 1; }
    $B $sh --opt $o --cold >> $O/times.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/times.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 tools/bench_pgemm.py fwd 32768 768 192 --reps 20 > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
find $O/pmc -name "*counter_collection.csv" | head -1 | xargs -I{} python3 -c "
import csv,collections,sys
rows=list(csv.DictReader(open('{}')))
agg=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in rows:
    k=r['Kernel_Name'][:60]; agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
for k,d in agg.items():
    print(k); print('   ', {c: round(v) for c,v in d.items()})
"
