set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/ab5; mkdir -p $O
V=krr_amd/lib/variants
L="$V/lib_z4.so $V/lib_o3z4.so $V/lib_o3z4f768.so $V/lib_o2c960.so"
for a in "--percentile 50" "--config 3 --containers 100000 --percentile 50" "--config 3 --containers 100000 --percentile 90" "--config 4 --containers 100000 --percentile 50"; do
  n=$(echo "$a" | tr -d ' -')
  timeout -k 10 300 python -u scripts/ab_variants.py $L $a > $O/$n.log 2>&1
  echo "== $a"; grep fused $O/$n.log
done
