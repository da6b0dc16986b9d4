set -e
cd ${GRAFT_REPO_ROOT:-/root/repo}
O=gpurun_out/ab1; mkdir -p $O
L="krr_amd/lib/variants/lib_base.so krr_amd/lib/variants/lib_o1d1.so krr_amd/lib/variants/lib_o1d2.so krr_amd/lib/variants/lib_o1d3.so krr_amd/lib/variants/lib_o2d2.so"
timeout -k 10 300 python -u scripts/ab_variants.py $L --percentile 99 > $O/c2p99.log 2>&1
timeout -k 10 300 python -u scripts/ab_variants.py $L --percentile 50 > $O/c2p50.log 2>&1
timeout -k 10 300 python -u scripts/ab_variants.py $L --config 3 --containers 100000 --percentile 50 > $O/c3p50.log 2>&1
timeout -k 10 300 python -u scripts/ab_variants.py $L --config 3 --containers 100000 --percentile 99 > $O/c3p99.log 2>&1
tail -n 6 $O/*.log
