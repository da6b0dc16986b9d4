#!/bin/bash
# PMC pass for config 2 p95 after the probe-backed single pass.
set -u -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/scripts/pmc_fetch.sh" c2_p95_v17 --config 2 --percentile 95 && echo pmc_v17 ok
