#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_strategy.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/t.log 2>&1 || { tail -30 gpurun_out/ab/t.log; exit 1; }
tail -1 gpurun_out/ab/t.log
V=krr_amd/lib/variants
timeout -k 10 400 python -u scripts/ab_variants.py $V/lib_lane0.so $V/lib_lane1.so $V/lib_lane0.so $V/lib_lane1.so --rounds 6 > gpurun_out/ab/ab.log 2>&1 || { tail -20 gpurun_out/ab/ab.log; exit 1; }
tail -4 gpurun_out/ab/ab.log
timeout -k 10 400 python -u scripts/ab_variants.py $V/lib_lane0.so $V/lib_lane1.so --rounds 4 --percentile 90 > gpurun_out/ab/ab90.log 2>&1 || { tail -20 gpurun_out/ab/ab90.log; exit 1; }
tail -2 gpurun_out/ab/ab90.log
timeout -k 10 400 python -u scripts/ab_variants.py $V/lib_lane0.so $V/lib_lane1.so --rounds 4 --config 3 > gpurun_out/ab/abc3.log 2>&1 || { tail -20 gpurun_out/ab/abc3.log; exit 1; }
tail -2 gpurun_out/ab/abc3.log
