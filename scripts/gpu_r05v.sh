set -o pipefail
mkdir -p gpurun_out/r05v
cat /sys/devices/system/node/node*/cpulist > gpurun_out/r05v/nodes.log 2>&1; cat /proc/self/status | grep -i cpus_allowed_list >> gpurun_out/r05v/nodes.log
timeout -k 10 300 python -u scripts/strip_pack_probe.py --only 1,256,1 > gpurun_out/r05v/strip_pack.log 2>&1 && \
timeout -k 10 300 python -u scripts/strip_pack_probe.py --only 1,256,1 --numa > gpurun_out/r05v/strip_pack_numa.log 2>&1 && \
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,10 > gpurun_out/r05v/hybrid.log 2>&1 && \
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,10 --numa > gpurun_out/r05v/hybrid_numa.log 2>&1
