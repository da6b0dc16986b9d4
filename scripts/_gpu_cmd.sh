#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_strategy.py tests/test_gpu_stress.py tests/test_gpu_sketch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/t.log 2>&1 || { tail -30 gpurun_out/ab/t.log; exit 1; }
tail -1 gpurun_out/ab/t.log
V=krr_amd/lib/variants
for c in "--mode ref_index" "--mode ref_index --percentile 50" "--mode ref_index --config 3"; do
timeout -k 10 400 python -u scripts/ab_variants.py $V/lib_old.so $V/lib_new.so $V/lib_old.so $V/lib_new.so --rounds 4 $c > gpurun_out/ab/ab.log 2>&1 || { tail -20 gpurun_out/ab/ab.log; exit 1; }
echo "== $c"; tail -2 gpurun_out/ab/ab.log
done
