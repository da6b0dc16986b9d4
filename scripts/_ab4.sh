set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/ab4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wselect.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
V=krr_amd/lib/variants
L="$V/lib_hsel.so $V/lib_f2304.so $V/lib_f1024.so $V/lib_f1024z4.so $V/lib_f512z4.so"
for a in "--percentile 50" "--config 3 --containers 100000 --percentile 50" "--config 3 --containers 100000 --percentile 90" "--config 3 --containers 100000 --percentile 75"; do
  n=$(echo "$a" | tr -d ' -')
  timeout -k 10 300 python -u scripts/ab_variants.py $L $a > $O/$n.log 2>&1
  echo "== $a"; grep fused $O/$n.log
done
for a in "--percentile 50 --containers 10000" "--percentile 50 --length 10080 --compact --containers 50000" "--percentile 50 --length 20160 --compact --containers 30000" "--percentile 50 --length 2880 --compact --containers 100000"; do
  n=$(echo "$a" | tr -d ' -')
  timeout -k 10 120 python -u scripts/diag_select.py $V/lib_diag_f1024.so $a > $O/diag_$n.log 2>&1
  echo "== diag $a"; grep -E "kernel|total|compact |final|n_compact|n_fallback|inserted|shares" $O/diag_$n.log
done
