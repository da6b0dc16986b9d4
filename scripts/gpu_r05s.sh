set -o pipefail
mkdir -p gpurun_out/r05s
for v in base nosev nodict o3 base; do
  timeout -k 10 200 python -u scripts/scan_probe.py krr_amd/lib/variants/pydec_$v >> gpurun_out/r05s/scan_probe.log 2>&1 || exit 1
done
