#!/bin/bash
# Round-end evidence for the current tree: smoke, GPU suite, default bench under rocprofv3
# kernel stats, and the p50 / p95 / ref_index / config-3 / config-4 lines.
set -u -o pipefail
TAG=${1:-v13}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
timeout -k 10 200 python -u __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo tests failed; tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 > "$OUT/c2.json" 2> "$OUT/c2.err") || { echo c2 failed; tail -20 "$OUT/c2.err"; exit 1; }
head -c 700 "$OUT/c2.json"; echo
for spec in "p50:--percentile 50" "p95:--percentile 95" "ref:--mode ref_index" "c3:--config 3" "c3p95:--config 3 --percentile 95" "c4:--config 4 --steps 3 --warmup 1" "c4p95:--config 4 --steps 3 --warmup 1 --percentile 95"; do
  name=${spec%%:*}; args=${spec#*:}
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline $args > "$OUT/$name.json" 2> "$OUT/$name.err") || { echo $name failed; tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']), d['ms_per_step'], d['kernels_ms'], round(d['roofline']['frac'],4))" "$OUT/$name.json" $name
done
echo v13 ok
