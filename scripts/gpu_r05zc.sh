set -o pipefail
mkdir -p gpurun_out/r05zc
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,10,12,14 --numa > gpurun_out/r05zc/hybrid_numa.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r05zc/bench.json 2> gpurun_out/r05zc/bench.err
