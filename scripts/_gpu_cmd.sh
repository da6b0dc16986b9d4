set -o pipefail
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_full.log 2>&1; rc=$?; tail -12 gpurun_out/gpu_tests_full.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/gpu_tests_full.log | head; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
