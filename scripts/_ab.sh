set -o pipefail
V=krr_amd/lib/variants
for c in "--config 2 --rounds 5 --percentile 94" "--config 2 --rounds 5 --percentile 93" "--config 2 --rounds 5 --percentile 95" "--config 2 --rounds 5 --percentile 92"; do
  echo "== $c"
  timeout -k 10 300 python -u scripts/ab_variants.py $V/lib_base.so $V/lib_c37.so $V/lib_c42.so $c || exit 1
done
