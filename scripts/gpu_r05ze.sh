set -o pipefail
mkdir -p gpurun_out/r05ze
V=krr_amd/lib/variants
timeout -k 10 400 python -u scripts/kll_sparse_probe.py $V/lib_runs0.so $V/lib_runs1.so $V/lib_check.so $V/lib_runs0.so $V/lib_runs1.so --check > gpurun_out/r05ze/runs.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kll.py > gpurun_out/r05ze/pytest_kll.log 2>&1
