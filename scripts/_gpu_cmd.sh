timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_h2.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_tests_h2.log; [ $rc -eq 0 ] || exit 1
V=krr_amd/lib/variants
for p in 99 95 90 75 50; do echo "p$p"; timeout -k 10 200 python -u scripts/ab_variants.py $V/lib_h2.so $V/lib_h3.so $V/lib_c4096.so --rounds 3 --percentile $p 2>&1 | grep -v amdgpu.ids || exit 1; done
