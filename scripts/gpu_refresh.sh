#!/bin/bash
# Refresh the bench lines + rocprofv3 kernel stats for every bench workload.
# usage: bash scripts/gpu_refresh.sh TAG
set -u -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# default bench line (config 2, linear p99) with CPU baseline, under rocprofv3 kernel stats
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 > "$OUT/c2.json" 2> "$OUT/c2.err") || { echo c2 failed; tail -20 "$OUT/c2.err"; exit 1; }
head -c 600 "$OUT/c2.json"; echo
for spec in "c3:--config 3" "c4:--config 4 --steps 3 --warmup 1" "ref:--mode ref_index" "p50:--percentile 50"; do
  name=${spec%%:*}; args=${spec#*:}
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline $args > "$OUT/$name.json" 2> "$OUT/$name.err") || { echo $name failed; tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['kernels_ms'], round(d['roofline']['frac'],4))" "$OUT/$name.json" $name
done
echo refresh ok
