set -o pipefail
mkdir -p gpurun_out/r05s
for v in base nosev nodict o3 base; do
  timeout -k 10 200 python -u scripts/scan_probe.py krr_amd/lib/variants/pydec_$v >> gpurun_out/r05s/scan_probe.log 2>&1 || exit 1
done
timeout -k 10 300 python -u scripts/strip_pack_probe.py --only 1,256,1 > gpurun_out/r05s/strip_pack.log 2>&1 && \
timeout -k 10 400 python -u scripts/hybrid_probe.py --strip 1 --dev-threads 8,10 > gpurun_out/r05s/hybrid_probe.log 2>&1
