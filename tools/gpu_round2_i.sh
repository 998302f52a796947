#!/bin/bash
# early exit of fully failed factorizations: bitwise fits/loop tests, then FHN-PDE / correction timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parareal.py tests/test_gpu_legacy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ri_tests.log 2>&1 || { tail -30 gpurun_out/ri_tests.log; exit 1; }
tail -2 gpurun_out/ri_tests.log
timeout -k 10 400 python -u tools/fhn_fits_probe.py 4 2>&1 | grep -v "amdgpu.ids" || exit 1
timeout -k 10 200 python -u tools/nm_probe.py 2>&1 | grep -v "^W20\|^E20\|amdgpu.ids" || exit 1
timeout -k 10 200 python -u tools/fhn_e2e.py 20 50 195325 2>&1 | grep "FHN-PDE" || exit 1
timeout -k 10 200 python -u tools/fhn_e2e.py 16 25 195325 2>&1 | grep "FHN-PDE" || exit 1
timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep early_stop || exit 1
