#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pipe
timeout -k 10 600 python -u scripts/bench_pipeline.py --objects 2000 --threads 16 > gpurun_out/pipe/p.json 2> gpurun_out/pipe/p.err || { tail -20 gpurun_out/pipe/p.err; exit 1; }
cat gpurun_out/pipe/p.json
