set -o pipefail
mkdir -p gpurun_out/r05h
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_json.py > gpurun_out/r05h/pytest_json.log 2>&1 && \
timeout -k 10 300 python -u scripts/kll_sparse_probe.py krr_amd/lib/variants/lib_pipe0.so krr_amd/lib/variants/lib_pipe1.so krr_amd/lib/variants/lib_pipe0.so krr_amd/lib/variants/lib_pipe1.so --check > gpurun_out/r05h/kll_pipe_probe.log 2>&1 && \
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 0,1 --dev-threads 4,6,8,10,12 > gpurun_out/r05h/hybrid_probe.log 2>&1
