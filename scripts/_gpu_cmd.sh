set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_p1.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests_p1.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/gpu_tests_p1.log | head; exit 1; }
timeout -k 10 300 python -u scripts/bench_pipeline.py --objects 2000 --threads 16 > gpurun_out/pipeline.json 2> gpurun_out/pipeline.err || { tail -20 gpurun_out/pipeline.err; exit 1; }
cat gpurun_out/pipeline.json
timeout -k 10 300 python -u scripts/bench_packer.py --threads 16 > gpurun_out/packer.json 2>&1; cat gpurun_out/packer.json
