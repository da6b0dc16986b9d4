#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, bench, rocprofv3 kernel-trace stats.
# Usage (from the repo root on the box): bash scripts/gpu_round.sh [tag] [bench args...]
set -u
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u __graft_entry__.py smoke > "$OUT/smoke_$TAG.log" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke_$TAG.log"; exit 1; }
tail -1 "$OUT/smoke_$TAG.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests_$TAG.log" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests_$TAG.log"
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "$OUT/gpu_tests_$TAG.log" | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 "$@" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || { tail -20 "$OUT/bench_$TAG.err"; exit 1; }
cat "$OUT/bench_$TAG.json"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$OUT/prof_$TAG.log" 2>&1 || { tail -20 "$OUT/prof_$TAG.log"; exit 1; }
find "$OUT/prof_$TAG" -name "*kernel_stats.csv" -exec cat {} \; | head -20
