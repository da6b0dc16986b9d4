#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/ov
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ov/bench.json 2> gpurun_out/ov/bench.err || { tail -20 gpurun_out/ov/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/ov/bench.json')); print(d['value'], d['ms_per_step'], d['kernels_ms'])"
KRR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --containers 2000 --steps 5 --warmup 1 > gpurun_out/ov/gloo2.json 2> gpurun_out/ov/gloo2.err || { grep -v Gloo gpurun_out/ov/gloo2.err | tail -30; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/ov/gloo2.json')); print(d['value'], d['ms_per_step'], d.get('parity_vs_oracle_on_sample'))"
