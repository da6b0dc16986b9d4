set -o pipefail
mkdir -p gpurun_out/r05u
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_json.py tests/test_gpu_strategy.py > gpurun_out/r05u/pytest.log 2>&1 && \
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,9,10 > gpurun_out/r05u/hybrid_probe.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r05u/bench.json 2> gpurun_out/r05u/bench.err
