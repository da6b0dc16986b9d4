set -o pipefail
mkdir -p gpurun_out/r05o
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/r05o/trace -o run -- python3 -u scripts/strip_pack_probe.py --only 1,256,1 > gpurun_out/r05o/trace.log 2>&1
