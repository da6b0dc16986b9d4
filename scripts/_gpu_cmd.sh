#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/st
timeout -k 10 400 python -u -m pytest tests/test_gpu_stress.py -x -v --timeout 120 --timeout-method thread > gpurun_out/st/t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/st/t.log | head -30; tail -2 gpurun_out/st/t.log; exit $rc
