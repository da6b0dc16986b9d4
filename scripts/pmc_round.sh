#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over scripts/profile_kernels.py.
# Usage: bash scripts/pmc_round.sh TAG [profile_kernels args...]
set -u
TAG=${1:-pmc}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $GROUP --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/scripts/profile_kernels.py" "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($GROUP) failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok: $GROUP"
done <<GROUPS
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH
FETCH_SIZE
WRITE_SIZE
GRBM_GUI_ACTIVE GRBM_COUNT
GROUPS
