set -o pipefail
V=krr_amd/lib/variants
for c in "--config 4 --containers 1000000 --rounds 3" "--config 2 --mode ref_index --rounds 9" "--config 2 --rounds 9" "--config 3 --containers 100000 --rounds 5"; do
  echo "== $c"
  timeout -k 10 300 python -u scripts/ab_variants.py $V/lib_base.so $V/lib_xcd.so $c || exit 1
done
