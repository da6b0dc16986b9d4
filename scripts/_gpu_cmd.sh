#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/c5d
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c5d/t.log 2>&1 || { tail -30 gpurun_out/c5d/t.log; exit 1; }
tail -1 gpurun_out/c5d/t.log
timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 > gpurun_out/c5d/full.json 2> gpurun_out/c5d/full.err || { tail -20 gpurun_out/c5d/full.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c5d/full.json')); print(round(d['value']), d['ms_per_step'], d['kernels_ms'], round(d['roofline']['frac'],3), d.get('parity_vs_single_window_select'), d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 300 python -u bench.py --percentile 97 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5d/p97.json 2> gpurun_out/c5d/p97.err || { tail -20 gpurun_out/c5d/p97.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c5d/p97.json')); print('p97', round(d['value']), d['ms_per_step'], d['kernels_ms'])"
