#!/bin/bash
# rocprofv3 kernel-trace stats + PMC FETCH/WRITE for the secondary workloads
# (hselect p50, config 3, config 5 sketch build).  usage: bash scripts/prof_round.sh TAG
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for spec in "p50:--percentile 50" "c3:--config 3" "c5:--config 5 --steps 3 --warmup 1"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${TAG}_$name" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline $args > "$OUT/prof_${TAG}_$name.log" 2>&1 || { echo "prof $name failed"; tail -5 "$OUT/prof_${TAG}_$name.log"; exit 1; }
  grep -h '"value"' "$OUT/prof_${TAG}_$name.log" | head -1 | cut -c1-400
  find "$OUT/prof_${TAG}_$name" -name "*kernel_stats.csv" -exec head -4 {} \;
done
cd "$R"
bash scripts/pmc_fetch.sh "fetch_${TAG}_p50" --percentile 50 || exit 1
bash scripts/pmc_fetch.sh "fetch_${TAG}_c5" --config 5 --containers 20000 || exit 1
python scripts/pmc_summary.py "$OUT/pmc_fetch_${TAG}_p50"
python scripts/pmc_summary.py "$OUT/pmc_fetch_${TAG}_c5"
