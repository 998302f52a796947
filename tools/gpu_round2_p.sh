#!/bin/bash
# select rewrite: kNN / predict / sweep parity tests, then the chain's per-phase clock on Burgers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parareal.py -m gpu -x -q --timeout 300 --timeout-method thread -k "knn or predict or fused_chain or speculative or bitwise_equals_oracle" > gpurun_out/rp_tests.log 2>&1 || { tail -40 gpurun_out/rp_tests.log; exit 1; }
tail -2 gpurun_out/rp_tests.log
bash tools/gpu_round2_o.sh
