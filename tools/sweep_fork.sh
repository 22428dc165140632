set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
B="timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity"
for rep in 1 2; do
for cfg in "default::" "nofork:OGV_FORK_MIN_WORK=1000000000000:" "nomb:: --opt mb_side=0" "none:OGV_FORK_MIN_WORK=1000000000000: --opt mb_side=0"; do
  name=${cfg%%:*}; rest=${cfg#*:}; envs=${rest%%:*}; opts=${rest#*:}
  out=$(env $envs $B $opts 2>&1 | grep -E '^\{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || { echo "$name failed"; exit 1; }
  echo "$name $out"
done
done
