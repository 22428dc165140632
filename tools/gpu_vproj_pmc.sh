#!/bin/bash
# SQ counters of the fused Outlooker forward vs the unfused pair (tools/bench_vproj.py), one PMC pass.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/vpmc; rm -rf $O; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_ANY SQ_INSTS_MFMA --output-format csv -d $O/pmc -o run -- python3 tools/bench_vproj.py --reps 3 > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
find $O/pmc -name "*counter_collection.csv" | head -1 | xargs -I{} python3 -c "
import csv,collections
rows=list(csv.DictReader(open('{}')))
agg=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in rows:
    k=r['Kernel_Name'][:70]; agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
for k,d in agg.items():
    print(k); print('   ', {c: round(v) for c,v in d.items()})
"
