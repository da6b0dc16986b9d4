set -o pipefail
mkdir -p gpurun_out/r05i /tmp/sb
g++ -O3 -std=c++17 -pthread -Ikrr_amd/csrc scripts/strip_bench.cpp -o /tmp/sb/sb1 && \
g++ -O3 -std=c++17 -pthread -Ikrr_amd/csrc -DKRR_STRIP_MASKED_STORES=0 scripts/strip_bench.cpp -o /tmp/sb/sb0 && \
timeout -k 10 120 /tmp/sb/sb1 > gpurun_out/r05i/strip_bench_masked.log 2>&1 && \
timeout -k 10 120 /tmp/sb/sb0 > gpurun_out/r05i/strip_bench_plain.log 2>&1 && \
lscpu > gpurun_out/r05i/lscpu.log 2>&1
