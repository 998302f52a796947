#!/bin/bash
# jitter-major rows in the speculative batch (Burgers / Hopf corrections)
set -o pipefail
mkdir -p gpurun_out
NNGP_NM_JMAJOR_SPEC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parareal.py -m gpu -x -q --timeout 300 --timeout-method thread -k "speculative or burgers or hopf" > gpurun_out/rm_tests.log 2>&1 || { tail -30 gpurun_out/rm_tests.log; exit 1; }
tail -1 gpurun_out/rm_tests.log
for jm in 0 1 0 1; do
  echo "== NNGP_NM_JMAJOR_SPEC=$jm"
  NNGP_NM_JMAJOR_SPEC=$jm timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep early_stop || exit 1
done
