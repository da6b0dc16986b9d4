#!/bin/bash
# Two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the fused kernel.
set -u
TAG=${1:-fetch}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/f" -o run -- python3 "$R/scripts/profile_kernels.py" "$@" > "$OUT/f.log" 2>&1 || { echo fetch pass failed; tail -5 "$OUT/f.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/w" -o run -- python3 "$R/scripts/profile_kernels.py" "$@" > "$OUT/w.log" 2>&1 || { echo write pass failed; tail -5 "$OUT/w.log"; exit 1; }
echo pmc ok
