set -o pipefail
mkdir -p gpurun_out/r05zd
V=krr_amd/lib/variants
timeout -k 10 400 python -u scripts/kll_sparse_probe.py $V/lib_base.so $V/lib_nl_ne.so $V/lib_nl_ne_nt.so > gpurun_out/r05zd/tau.log 2>&1
