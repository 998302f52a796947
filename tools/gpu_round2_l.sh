#!/bin/bash
# jitter-major fit assignment in the packed kernel: bitwise tests with it forced, then FHN timings
set -o pipefail
mkdir -p gpurun_out
NNGP_NM_JMAJOR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -k "predict or nm_" > gpurun_out/rl_tests.log 2>&1 || { tail -30 gpurun_out/rl_tests.log; exit 1; }
tail -1 gpurun_out/rl_tests.log
for jm in 0 1; do
  echo "== NNGP_NM_JMAJOR=$jm"
  NNGP_NM_JMAJOR=$jm timeout -k 10 300 python -u tools/fhn_fits_probe.py 4 2>&1 | grep "slice" || exit 1
  NNGP_NM_JMAJOR=$jm timeout -k 10 200 python -u tools/nm_probe.py 2>&1 | grep "d= 800" || exit 1
done
