set -o pipefail
mkdir -p gpurun_out/r05p
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_json.py > gpurun_out/r05p/pytest_json.log 2>&1 && \
timeout -k 10 300 python -u scripts/strip_pack_probe.py --only 1,256,1 > gpurun_out/r05p/strip_pack.log 2>&1 && \
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,10,12,13 > gpurun_out/r05p/hybrid_probe.log 2>&1
