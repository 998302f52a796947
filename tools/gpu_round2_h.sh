#!/bin/bash
# FHN-PDE point-pair field kernel: bitwise tests, then per-step times with it and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_contract.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fhn or field or rk_ or contract" > gpurun_out/rh_tests.log 2>&1 || { tail -30 gpurun_out/rh_tests.log; exit 1; }
tail -2 gpurun_out/rh_tests.log
for pr in 1 0; do
  echo "== NNGP_FHN_PAIR=$pr"
  NNGP_FHN_PAIR=$pr timeout -k 10 300 python -u tools/contract_probe.py 2>&1 | grep fhn || exit 1
done
timeout -k 10 200 python -u tools/fhn_e2e.py 20 50 195325 2>&1 | grep "FHN-PDE" || exit 1
