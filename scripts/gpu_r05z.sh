set -o pipefail
mkdir -p gpurun_out/r05za
V=krr_amd/lib/variants
timeout -k 10 400 python -u scripts/kll_sparse_probe.py $V/lib_ex0.so $V/lib_ex1.so $V/lib_ex0.so $V/lib_ex1.so --check > gpurun_out/r05za/export.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kll.py > gpurun_out/r05za/pytest_kll.log 2>&1
