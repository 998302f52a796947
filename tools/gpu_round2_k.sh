#!/bin/bash
# new parity tests: TomLab N=256 oracle loop, multi-rank (gloo, shared GPU) runs with the HIP path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parareal.py tests/test_gpu_distributed.py -m gpu -v --timeout 400 --timeout-method thread -k "tomlab or multi_rank" > gpurun_out/rk_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/rk_tests.log | tail -15
exit $rc
