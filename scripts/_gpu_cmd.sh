#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/d
T="timeout -k 10 240"
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
$T python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/d/n1.json 2> gpurun_out/d/n1.err || { tail gpurun_out/d/n1.err; exit 1; }
p=29620
for g in pipelined blocking; do
  p=$((p+1))
  $T $TR --master-port $p bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-dist --gather $g > gpurun_out/d/fd_$g.json 2> gpurun_out/d/fd_$g.err || { tail gpurun_out/d/fd_$g.err; exit 1; }
done
KRR_BENCH_BACKEND=gloo $T python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --steps 5 --warmup 1 --no-cpu-baseline --containers 2000 > gpurun_out/d/gloo2.json 2> gpurun_out/d/gloo2.err || { tail gpurun_out/d/gloo2.err; exit 1; }
for f in n1 fd_pipelined fd_blocking gloo2; do wc -l < gpurun_out/d/$f.json; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['n_gpus'], round(d['value']), d['ms_per_step'], d['kernels_ms'])" gpurun_out/d/$f.json $f; done
