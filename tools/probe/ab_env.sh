# Same-box A/B of an environment switch on bench_configs:
#   bash tools/probe/ab_env.sh <tag> <configs> "<VAR=value ...>"   (the first run of each pair has no switch)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
for i in 1 2; do
  for v in off on; do
    envs=""; [ $v = on ] && envs="$3"
    env $envs timeout -k 10 300 python -u tools/bench_configs.py --reps 3 --no-host --configs "$2" \
      > "$OUT/ab_${v}_$i.log" 2>&1 || exit 3
    echo "$v #$i: $(grep -h '^{"configs"' "$OUT/ab_${v}_$i.log" | cut -c1-600)"
  done
done
