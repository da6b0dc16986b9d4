#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/t
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t/t.log 2>&1 || { tail -30 gpurun_out/t/t.log; exit 1; }
tail -1 gpurun_out/t/t.log
bash scripts/gpu_refresh.sh "$1"
