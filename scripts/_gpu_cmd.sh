#!/bin/bash
# final-evidence pass: PMC traffic of the default bench kernel, then the bench line under rocprofv3 stats
set -o pipefail
TAG=$1
bash scripts/pmc_fetch.sh "fetch_config2_linear_$TAG" || exit 1
python scripts/pmc_traffic.py "gpurun_out/pmc_fetch_config2_linear_$TAG" "config2:linear:p99:k_simple" 10000 || exit 1
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash scripts/gpu_refresh.sh "$TAG"
