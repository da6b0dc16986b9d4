#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/diag
timeout -k 10 200 python -u scripts/diag_select.py krr_amd/lib/variants/lib_diag.so > gpurun_out/diag/c2.log 2>&1 || { tail -20 gpurun_out/diag/c2.log; exit 1; }
cat gpurun_out/diag/c2.log | grep -v amdgpu.ids
timeout -k 10 200 python -u scripts/diag_select.py krr_amd/lib/variants/lib_diag.so --length 10080 --compact --containers 200000 > gpurun_out/diag/c4.log 2>&1 || { tail -20 gpurun_out/diag/c4.log; exit 1; }
cat gpurun_out/diag/c4.log | grep -v amdgpu.ids
