#!/bin/bash
# GPU: same-process timing of the KLL build variants in krr_amd/lib/variants (tail 0 and TAIL),
# then one SQ counter pass per variant and tail (SQ_TAILS, default TAIL).
# usage: [SQ_TAILS="0 1792"] bash scripts/kll_variants.sh TAG [TAIL] [SERIES]
set -u
TAG=${1:?tag}; TAIL=${2:-1792}; SER=${3:-20000}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
LIBS=$(ls krr_amd/lib/variants/lib_*.so)
for t in 0 $TAIL; do
  timeout -k 10 300 python -u scripts/kll_probe.py $LIBS --series $SER --tail $t > "$OUT/probe_t$t.log" 2>&1 \
    || { echo "probe failed"; tail "$OUT/probe_t$t.log"; exit 1; }
  grep median "$OUT/probe_t$t.log"
done
for L in $LIBS; do
  n=$(basename $L .so)
  for t in ${SQ_TAILS:-$TAIL}; do
    timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY \
      --output-format csv -d "$OUT/sq_${n}_t$t" -o run -- python3 scripts/kll_probe.py $L --series $SER --tail $t --rounds 1 \
      > "$OUT/sq_${n}_t$t.log" 2>&1 || { echo "sq $n failed"; tail "$OUT/sq_${n}_t$t.log"; exit 1; }
    echo "== $n tail $t"; python3 scripts/pmc_summary.py "$OUT/sq_${n}_t$t" | grep -A9 kll_build
  done
done
