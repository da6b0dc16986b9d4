set -o pipefail
mkdir -p gpurun_out/r05j
timeout -k 10 500 python -u scripts/strip_pack_probe.py > gpurun_out/r05j/strip_pack_probe.log 2>&1
