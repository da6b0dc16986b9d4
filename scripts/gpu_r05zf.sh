set -o pipefail
mkdir -p gpurun_out/r05zf /tmp/sb
g++ -O3 -std=c++17 -pthread -Ikrr_amd/csrc scripts/strip_bench.cpp -o /tmp/sb/sb && \
timeout -k 10 200 /tmp/sb/sb > gpurun_out/r05zf/strip_bench_all.log 2>&1 && \
timeout -k 10 200 taskset -c $(cat /sys/devices/system/node/node0/cpulist) /tmp/sb/sb > gpurun_out/r05zf/strip_bench_node0.log 2>&1
