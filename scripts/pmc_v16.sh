#!/bin/bash
# PMC refresh after the select probe: config 2 p99, config 3 p99 / p95.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/scripts/pmc_fetch.sh" c2_p99_v16 --config 2 --percentile 99 \
 && bash "$R/scripts/pmc_fetch.sh" c3_p99_v16 --config 3 --containers 100000 \
 && bash "$R/scripts/pmc_fetch.sh" c3_p95_v16 --config 3 --containers 100000 --percentile 95 \
 && echo pmc_v16 ok
