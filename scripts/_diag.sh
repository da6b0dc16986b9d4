set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/diag1; mkdir -p $O
V=krr_amd/lib/variants
for a in "--percentile 50 --containers 10000" "--percentile 50 --length 10080 --compact --containers 50000" "--percentile 50 --length 20160 --compact --containers 30000" "--percentile 50 --length 2880 --compact --containers 100000" "--percentile 90 --length 10080 --compact --containers 50000" "--percentile 99 --length 10080 --compact --containers 50000"; do
  n=$(echo "$a" | tr -d ' -')
  timeout -k 10 120 python -u scripts/diag_select.py $V/lib_diag.so $a > $O/diag_$n.log 2>&1
  echo "== diag $a"; grep -E "kernel|total|compact |final|n_compact|n_fallback|inserted|shares" $O/diag_$n.log
done
