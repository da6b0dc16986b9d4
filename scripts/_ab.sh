set -o pipefail
V=krr_amd/lib/variants
for c in "--config 3 --containers 100000 --percentile 95 --rounds 7" "--config 3 --containers 100000 --rounds 7" "--config 2 --rounds 7"; do
  echo "== $c"
  timeout -k 10 300 python -u scripts/ab_variants.py $V/lib_base.so $V/lib_w2.so $c || exit 1
done
