#!/bin/bash
# PMC refresh (FETCH_SIZE / WRITE_SIZE passes) of the fused kernel on the current tree:
# config 2 at p99 / p95 / p50 and ref_index, config 3 at p99 / p95.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/scripts/pmc_fetch.sh" c2_p99_v14 --config 2 --percentile 99 \
 && bash "$R/scripts/pmc_fetch.sh" c2_p95_v14 --config 2 --percentile 95 \
 && bash "$R/scripts/pmc_fetch.sh" c2_p50_v14 --config 2 --percentile 50 \
 && bash "$R/scripts/pmc_fetch.sh" c2_ref_v14 --config 2 --mode ref_index \
 && bash "$R/scripts/pmc_fetch.sh" c3_p99_v14 --config 3 --containers 100000 \
 && bash "$R/scripts/pmc_fetch.sh" c3_p95_v14 --config 3 --containers 100000 --percentile 95 \
 && echo pmc_v14 ok
