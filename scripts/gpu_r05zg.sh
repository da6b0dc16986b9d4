set -o pipefail
mkdir -p gpurun_out/r05zg /tmp/sb
g++ -O3 -std=c++17 -pthread -Ikrr_amd/csrc scripts/strip_bench.cpp -o /tmp/sb/sb_nt && \
g++ -O3 -std=c++17 -pthread -Ikrr_amd/csrc -DKRR_STRIP_NT=0 scripts/strip_bench.cpp -o /tmp/sb/sb_plain && \
timeout -k 10 200 taskset -c $(cat /sys/devices/system/node/node0/cpulist) /tmp/sb/sb_plain > gpurun_out/r05zg/plain.log 2>&1 && \
timeout -k 10 200 taskset -c $(cat /sys/devices/system/node/node0/cpulist) /tmp/sb/sb_nt > gpurun_out/r05zg/nt.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_json.py > gpurun_out/r05zg/pytest_json.log 2>&1 && \
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 10,12 --numa > gpurun_out/r05zg/hybrid.log 2>&1
