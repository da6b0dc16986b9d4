set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; export TMPDIR=/tmp
OUT=$R/gpurun_out/r04/b; mkdir -p $OUT
L=krr_amd/lib/libkrr_amd.so
timeout -k 10 200 python -u scripts/kll_probe.py $L --series 20000 --tail 1792 > $OUT/probe_t1792.log 2>&1 || { tail $OUT/probe_t1792.log; exit 1; }
timeout -k 10 200 python -u scripts/kll_probe.py $L --series 20000 --tail 0 > $OUT/probe_t0.log 2>&1 || { tail $OUT/probe_t0.log; exit 1; }
cat $OUT/probe_*.log
i=0
for cs in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
          "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $cs --output-format csv -d $OUT/sq_$i -o run -- python3 scripts/kll_probe.py $L --series 20000 --tail 1792 --rounds 1 > $OUT/sq_$i.log 2>&1 || { echo "sq $i failed"; tail $OUT/sq_$i.log; exit 1; }
done
python3 scripts/pmc_summary.py $OUT > $OUT/sq.txt 2>&1; cat $OUT/sq.txt | head -40
