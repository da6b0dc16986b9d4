set -o pipefail
mkdir -p gpurun_out/r05zi
V=krr_amd/lib/variants
timeout -k 10 400 python -u scripts/kll_sparse_probe.py $V/lib_lc0.so $V/lib_lc1.so $V/lib_lc0.so $V/lib_lc1.so --check > gpurun_out/r05zi/levelcopy.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kll.py > gpurun_out/r05zi/pytest_kll.log 2>&1
