set -o pipefail
mkdir -p gpurun_out/r05r
V=krr_amd/lib/variants
timeout -k 10 400 python -u scripts/kll_sparse_probe.py $V/lib_base.so $V/lib_noexport.so $V/lib_nofilter.so $V/lib_noload.so $V/lib_noload_noexport.so $V/lib_base.so > gpurun_out/r05r/tail_parts.log 2>&1
