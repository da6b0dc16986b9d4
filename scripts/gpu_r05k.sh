set -o pipefail
mkdir -p gpurun_out/r05k
timeout -k 10 600 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,12,14 --fixed-shares 0.02,0.06,0.1,0.14 > gpurun_out/r05k/hybrid_fixed.log 2>&1
