#!/bin/bash
# Round pass 2: standard round (smoke, tests, bench config 2, rocprof stats), PMC
# FETCH/WRITE of the fused kernel, then the other workloads' bench lines.
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
cd "$R"
bash scripts/gpu_round.sh "$TAG" || exit 1
bash scripts/pmc_fetch.sh "fetch_$TAG" || exit 1
for args in "--config 3" "--config 4" "--mode sorted_lower" "--mode ref_index" "--percentile 50" "--percentile 90"; do
  name=$(echo "$args" | tr -d ' -')
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline $args > "$OUT/bench_${TAG}_$name.json" 2> "$OUT/bench_${TAG}_$name.err" || { echo "bench $args failed"; tail -5 "$OUT/bench_${TAG}_$name.err"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['kernels_ms'], round(d['roofline']['frac'],3))" "$OUT/bench_${TAG}_$name.json" "$args"
done
