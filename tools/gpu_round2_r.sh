#!/bin/bash
# threshold select: parity tests, then chain phases with 8 workgroups and with 1, and the unfused A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parareal.py -m gpu -x -q --timeout 300 --timeout-method thread -k "knn or predict or fused_chain or speculative or bitwise_equals_oracle" > gpurun_out/rr_tests.log 2>&1 || { tail -40 gpurun_out/rr_tests.log; exit 1; }
tail -1 gpurun_out/rr_tests.log
echo "== 8 WGs"; bash tools/gpu_round2_o.sh || exit 1
echo "== 1 WG"; NNGP_CHAIN_WGS=1 bash tools/gpu_round2_o.sh || exit 1
echo "== unfused"; NNGP_CHAIN=0 timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep early_stop
