#!/bin/bash
# scratch: config-5 exact bench + rocprofv3 kernel stats
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/c5x
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 > gpurun_out/c5x/bench.json 2> gpurun_out/c5x/bench.err || { tail -20 gpurun_out/c5x/bench.err; exit 1; }
cat gpurun_out/c5x/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/c5x/prof" -o run -- python3 "$R/bench.py" --config 5 --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/c5x/prof.log" 2>&1 || { tail -20 "$R/gpurun_out/c5x/prof.log"; exit 1; }
find "$R/gpurun_out/c5x/prof" -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -12
