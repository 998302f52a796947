#!/bin/bash
# split re-speculation window: parity (speculative sweep tests), then Burgers / Hopf-shaped A/B
set -o pipefail
mkdir -p gpurun_out
NNGP_RESPEC_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parareal.py -m gpu -x -q --timeout 300 --timeout-method thread -k "speculative or bitwise or burgers or fused_chain" > gpurun_out/rv_tests.log 2>&1 || { tail -40 gpurun_out/rv_tests.log; exit 1; }
tail -1 gpurun_out/rv_tests.log
for sp in 0 1 0 1; do echo "== NNGP_RESPEC_SPLIT=$sp"; NNGP_RESPEC_SPLIT=$sp timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep "early_stop=None" || exit 1; done
