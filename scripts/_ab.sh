set -o pipefail
V=krr_amd/lib/variants
for c in "--config 2 --rounds 5 --percentile 50" "--config 2 --rounds 5 --percentile 75" "--config 2 --rounds 5 --percentile 90" "--config 3 --containers 100000 --percentile 50 --rounds 5" "--config 3 --containers 100000 --percentile 90 --rounds 5"; do
  echo "== $c"
  timeout -k 10 300 python -u scripts/ab_variants.py $V/lib_base.so $V/lib_h9.so $V/lib_h8.so $c || exit 1
done
