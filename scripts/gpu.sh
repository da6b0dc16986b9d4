#!/bin/bash
# One GPU-box pass, parameterised (replaces the per-version launchers of round 1).
#   bash scripts/gpu.sh TAG STEP...
# steps:
#   tests        pytest -m gpu (one process, per-test timeout) + smoke()
#   tests:EXPR   only the GPU tests matching -k EXPR
#   bench        bench.py default (config 2, linear p99) -> bench.json
#   bench:ARGS   bench.py with ARGS (commas for spaces), e.g. bench:--config,3
#   prof         rocprofv3 --kernel-trace --stats of the default bench -> kernel_stats.csv
#   prof:ARGS    the same for bench.py ARGS
#   pmc          FETCH_SIZE / WRITE_SIZE passes of the default bench (separate runs)
#   pmc:ARGS     the same for bench.py ARGS
#   ab:ARGS      same-process A/B of every krr_amd/lib/variants/lib_*.so (scripts/build_variants.sh)
#                on the ab_variants.py workload ARGS, e.g. ab:--config,3,--percentile,50
#   sq:ARGS      SQ issue / wait counters (two rocprofv3 --pmc passes) of the ab_variants.py workload
#   script:NAME,ARGS  python scripts/NAME.py ARGS -> script_NAME_ARGS.log
#   sqs:NAME,ARGS  the sq counter passes over python scripts/NAME.py LIB ARGS (e.g. kll_sparse_probe)
#   diag:ARGS    per-segment phase breakdown with krr_amd/lib/variants/lib_diag.so (-DKRR_DIAG)
# Every GPU step runs under its own timeout; the first failure ends the script.
set -u
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
export TMPDIR=/tmp

name_of() { echo "$1" | tr -d ' -' | tr ',' '_' | tr '=' '_'; }

for step in "$@"; do
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  args=${arg//,/ }
  n=$(name_of "$arg")
  case "$kind" in
    tests)
      sel=()
      [[ -n "$arg" ]] && sel=(-k "$args")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${sel[@]}" \
        > "$OUT/pytest${n:+_$n}.log" 2>&1 || { echo "gpu tests failed"; tail -40 "$OUT/pytest${n:+_$n}.log"; exit 1; }
      tail -3 "$OUT/pytest${n:+_$n}.log"
      if [[ -z "$arg" ]]; then
        timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
          || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
        tail -1 "$OUT/smoke.log"
      fi
      ;;
    bench)
      timeout -k 10 600 python -u bench.py $args > "$OUT/bench${n:+_$n}.json" 2> "$OUT/bench${n:+_$n}.err" \
        || { echo "bench $args failed"; tail -20 "$OUT/bench${n:+_$n}.err"; exit 1; }
      python - "$OUT/bench${n:+_$n}.json" "$args" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2] or "default", "value", round(d["value"]), "ms", round(d["ms_per_step"], 4), "kernels", d.get("kernels_ms"),
      "frac", round(d["roofline"]["frac"], 4), "parity", d.get("parity_vs_oracle_on_sample"))
EOF
      ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof${n:+_$n}" -o run -- \
        python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline $args > "$OUT/prof${n:+_$n}.log" 2>&1 \
        || { echo "prof $args failed"; tail -20 "$OUT/prof${n:+_$n}.log"; exit 1; }
      f=$(find "$OUT/prof${n:+_$n}" -name '*kernel_stats.csv' | head -1)
      cp "$f" "$OUT/kernel_stats${n:+_$n}.csv"
      head -4 "$OUT/kernel_stats${n:+_$n}.csv" | cut -c1-200
      ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc "$c" --output-format csv -d "$OUT/pmc${n:+_$n}_$c" -o run -- \
          python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $args > "$OUT/pmc${n:+_$n}_$c.log" 2>&1 \
          || { echo "pmc $c $args failed"; tail -20 "$OUT/pmc${n:+_$n}_$c.log"; exit 1; }
      done
      ;;
    ab)
      libs=$(ls krr_amd/lib/variants/lib_*.so | grep -v lib_diag)
      timeout -k 10 300 python -u scripts/ab_variants.py $libs $args > "$OUT/ab${n:+_$n}.log" 2>&1 \
        || { echo "ab $args failed"; tail -20 "$OUT/ab${n:+_$n}.log"; exit 1; }
      echo "== ab $args"; grep fused "$OUT/ab${n:+_$n}.log"
      ;;
    script)
      # script:NAME,ARGS  python -u scripts/NAME.py ARGS (under its own 300-s limit)
      sname=${args%% *}
      sargs=""
      [[ "$args" == *" "* ]] && sargs=${args#* }
      timeout -k 10 300 python -u "scripts/$sname.py" $sargs > "$OUT/script_${n}.log" 2>&1 \
        || { echo "script $args failed"; tail -20 "$OUT/script_${n}.log"; exit 1; }
      echo "== script $args"; tail -5 "$OUT/script_${n}.log"
      ;;
    diag)
      timeout -k 10 120 python -u scripts/diag_select.py krr_amd/lib/variants/lib_diag.so $args \
        > "$OUT/diag${n:+_$n}.log" 2>&1 || { echo "diag $args failed"; tail -20 "$OUT/diag${n:+_$n}.log"; exit 1; }
      echo "== diag $args"; grep -E "kernel|total|compact |final|n_compact|n_fallback|inserted|shares" "$OUT/diag${n:+_$n}.log"
      ;;
    sq)
      # SQ issue / wait counters of every kernel of the ab_variants.py workload ARGS, run on
      # the in-tree library (SQLIB overrides); two separate passes (8 SQ counters each at most)
      lib=${SQLIB:-krr_amd/lib/libkrr_amd.so}
      i=0
      for cs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
                "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC"; do
        i=$((i + 1))
        timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d "$OUT/sq${n:+_$n}_$i" -o run -- \
          python3 scripts/ab_variants.py $lib $args --rounds 2 > "$OUT/sq${n:+_$n}_$i.log" 2>&1 \
          || { echo "sq pass $i $args failed"; tail -20 "$OUT/sq${n:+_$n}_$i.log"; exit 1; }
      done
      python3 scripts/pmc_summary.py "$OUT" > "$OUT/sq${n:+_$n}.txt" 2>&1 && cat "$OUT/sq${n:+_$n}.txt"
      ;;
    sqs)
      # SQ counters of every kernel of scripts/NAME.py LIB ARGS (two passes of 8 SQ counters)
      lib=${SQLIB:-krr_amd/lib/libkrr_amd.so}
      sname=${args%% *}
      sargs=""
      [[ "$args" == *" "* ]] && sargs=${args#* }
      i=0
      for cs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
                "SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM"; do
        i=$((i + 1))
        timeout -s KILL 150 rocprofv3 --pmc $cs --output-format csv -d "$OUT/sqs${n:+_$n}_$i" -o run -- \
          python3 "scripts/$sname.py" $lib $sargs > "$OUT/sqs${n:+_$n}_$i.log" 2>&1 \
          || { echo "sqs pass $i $args failed"; tail -20 "$OUT/sqs${n:+_$n}_$i.log"; exit 1; }
      done
      python3 scripts/pmc_summary.py "$OUT" > "$OUT/sqs${n:+_$n}.txt" 2>&1 && cat "$OUT/sqs${n:+_$n}.txt"
      ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu.sh $TAG done"
