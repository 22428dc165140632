#!/bin/bash
# Two separate rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE cannot share one pass on gfx950) over
# a short eager bench run, then per-launch HBM traffic of the roofline kernels.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
rm -rf "$OUT"; mkdir -p "$OUT"
ARGS="--eager --steps 2 --warmup 1 --no-cpu-baseline --no-parity"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $ARGS > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || exit $?
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" --out "$OUT/pmc_traffic.json"
find "$OUT" -name "*counter_collection.csv" -exec gzip -f {} \;
find "$OUT" -type f ! -name "*.gz" ! -name "*.json" ! -name "*.log" -delete   # stay under gpurun's 64 MiB merge cap
du -sh "$OUT"
