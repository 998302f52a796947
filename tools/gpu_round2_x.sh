#!/bin/bash
# overlapped speculative batch: parity, then Burgers / chain-probe A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parareal.py tests/test_gpu_distributed.py tests/test_gpu_legacy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rx_tests.log 2>&1 || { tail -40 gpurun_out/rx_tests.log; exit 1; }
tail -1 gpurun_out/rx_tests.log
for ov in 0 1 0 1; do echo "== NNGP_SPEC_OVERLAP=$ov"; NNGP_SPEC_OVERLAP=$ov timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep "early_stop=None" || exit 1; done
