set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_s1.log 2>&1; rc=$?; tail -15 gpurun_out/gpu_tests_s1.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py --config 5 --containers 2000 --steps 3 --warmup 1 > gpurun_out/bench_c5_small.json 2> gpurun_out/bench_c5_small.err || { tail -20 gpurun_out/bench_c5_small.err; exit 1; }
cat gpurun_out/bench_c5_small.json
KRR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --config 5 --containers 2000 --steps 3 --warmup 1 > gpurun_out/bench_c5_gloo2.json 2> gpurun_out/bench_c5_gloo2.err || { tail -20 gpurun_out/bench_c5_gloo2.err; exit 1; }
cat gpurun_out/bench_c5_gloo2.json
timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -20 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
