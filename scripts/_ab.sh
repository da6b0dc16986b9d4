set -o pipefail
V=krr_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "probe_start or random_ragged or hselect or long_series" || exit 1
for c in "--config 3 --containers 100000 --percentile 95 --rounds 5" "--config 2 --rounds 5" "--config 3 --containers 100000 --rounds 5" "--config 4 --containers 100000 --percentile 95 --rounds 5" "--config 4 --containers 100000 --rounds 5" "--config 3 --containers 100000 --percentile 97 --rounds 5"; do
  echo "== $c"
  timeout -k 10 300 python -u scripts/ab_variants.py $V/lib_base.so $V/lib_probe.so $V/lib_probe1.so $V/lib_probe15.so $V/lib_probe3.so $c || exit 1
done
