set -o pipefail
V=krr_amd/lib/variants
for c in "--config 2 --rounds 5" "--config 4 --containers 100000 --rounds 5" "--config 3 --containers 100000 --percentile 99 --rounds 5" "--config 3 --containers 100000 --percentile 95 --rounds 5" "--config 4 --containers 100000 --percentile 98 --rounds 5" "--config 2 --rounds 5 --mode sorted_lower"; do
  echo "== $c"
  timeout -k 10 300 python -u scripts/ab_variants.py $V/lib_base.so $V/lib_g05.so $V/lib_g025.so $V/lib_g0.so $c || exit 1
done
