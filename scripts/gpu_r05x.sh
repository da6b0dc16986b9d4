set -o pipefail
mkdir -p gpurun_out/r05x
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,9,10 --numa > gpurun_out/r05x/hybrid_numa.log 2>&1 && \
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,9,10 --numa --cores > gpurun_out/r05x/hybrid_numa_cores.log 2>&1
