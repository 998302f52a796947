#!/bin/bash
# wave-wide fits kernel: bitwise tests, then correction / FHN e2e / Burgers timings (default policy
# and NNGP_NM_WAVE=0, the round-1 kernels)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -k "predict or nm_ or knn or gp_mean" > gpurun_out/rd_tests.log 2>&1 || { tail -30 gpurun_out/rd_tests.log; exit 1; }
tail -2 gpurun_out/rd_tests.log
for w in -1 0; do
  echo "== NNGP_NM_WAVE=$w"
  NNGP_NM_WAVE=$w timeout -k 10 200 python -u tools/nm_probe.py 2>&1 | grep -v "^W20\|^E20\|amdgpu.ids" || exit 1
  NNGP_NM_WAVE=$w timeout -k 10 200 python -u tools/fhn_e2e.py 20 50 195325 2>&1 | grep "FHN-PDE" || exit 1
  NNGP_NM_WAVE=$w timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep early_stop || exit 1
done
