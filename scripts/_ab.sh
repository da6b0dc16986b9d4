set -o pipefail
V=krr_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "probe or hselect or long_series" || exit 1
for c in "--config 2 --rounds 5 --percentile 95" "--config 2 --rounds 5 --percentile 97" "--config 3 --containers 100000 --percentile 90 --rounds 5" "--config 2 --rounds 5 --percentile 96" "--config 2 --rounds 5 --percentile 94"; do
  echo "== $c"
  timeout -k 10 300 python -u scripts/ab_variants.py $V/lib_base.so $V/lib_new.so $c || exit 1
done
