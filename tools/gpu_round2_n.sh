#!/bin/bash
# fused correction chain: A/B parity tests, the speculative-sweep tests, then Burgers wall-clock A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parareal.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "fused_chain or speculative or bitwise_equals_oracle" > gpurun_out/rn_tests.log 2>&1 || { tail -40 gpurun_out/rn_tests.log; exit 1; }
grep -E "passed|failed|chain launches" gpurun_out/rn_tests.log | tail -12
for ch in 0 1 0 1; do
  echo "== NNGP_CHAIN=$ch"
  NNGP_CHAIN=$ch timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep early_stop || exit 1
done
