set -o pipefail
V=krr_amd/lib/variants
timeout -k 10 200 python -u scripts/ab_variants.py $V/lib_d1.so $V/lib_d2.so --rounds 7 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -u scripts/ab_variants.py $V/lib_d1.so $V/lib_d2.so --rounds 5 --config 3 --containers 100000 2>&1 | grep -v amdgpu.ids || exit 1
