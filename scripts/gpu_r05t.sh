set -o pipefail
mkdir -p gpurun_out/r05t
for v in noproto base noproto base; do
  timeout -k 10 200 python -u scripts/scan_probe.py krr_amd/lib/variants/pydec_$v >> gpurun_out/r05t/scan_probe.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py > gpurun_out/r05t/bench.json 2> gpurun_out/r05t/bench.err
