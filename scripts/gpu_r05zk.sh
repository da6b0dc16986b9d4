set -o pipefail
mkdir -p gpurun_out/r05zk
for c in 256 512 1024 256 512 1024; do
  timeout -k 10 200 python -u scripts/strip_pack_probe.py --numa --only 1,$c,1 >> gpurun_out/r05zk/chunks.log 2>&1 || exit 1
done
