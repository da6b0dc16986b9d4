set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/ab12; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wselect.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
V=krr_amd/lib/variants
L="$V/lib_prev.so $V/lib_new.so"
for a in "--percentile 50" "--percentile 99" "--config 3 --containers 100000 --percentile 50" "--config 3 --containers 100000 --percentile 90" "--config 3 --containers 100000 --percentile 99" "--percentile 90" "--percentile 75" "--config 4 --containers 100000 --percentile 50"; do
  n=$(echo "$a" | tr -d ' -')
  timeout -k 10 300 python -u scripts/ab_variants.py $L $a > $O/$n.log 2>&1
  echo "== $a"; grep fused $O/$n.log
done
