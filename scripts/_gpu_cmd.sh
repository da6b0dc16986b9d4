#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ab
for k in 1 2; do
for f in "" "--serial-copy"; do
timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline $f > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -20 gpurun_out/ab/b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/ab/b.json')); print('$f', d['ms_per_step'], d['kernels_ms'], d['value'])"
done
done
