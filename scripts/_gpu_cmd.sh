#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab
V=krr_amd/lib/variants
for c in "--config 2" "--config 3" "--config 4 --containers 100000" "--config 2 --mode sorted_lower"; do
timeout -k 10 400 python -u scripts/ab_variants.py $V/lib_slack0.so $V/lib_slack.so $V/lib_slack0.so $V/lib_slack.so --rounds 4 $c > gpurun_out/ab/ab.log 2>&1 || { tail -20 gpurun_out/ab/ab.log; exit 1; }
echo "== $c"; tail -2 gpurun_out/ab/ab.log
done
