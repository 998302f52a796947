#!/bin/bash
# 32-lane fits for m = 17..32: bitwise kernel + loop tests, then correction / FHN e2e / Burgers timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parareal.py tests/test_gpu_legacy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/re_tests.log 2>&1 || { tail -30 gpurun_out/re_tests.log; exit 1; }
tail -2 gpurun_out/re_tests.log
timeout -k 10 200 python -u tools/nm_probe.py 2>&1 | grep -v "^W20\|^E20\|amdgpu.ids" || exit 1
timeout -k 10 200 python -u tools/fhn_e2e.py 20 50 195325 2>&1 | grep "FHN-PDE" || exit 1
timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep early_stop || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fhn_e2e_b -o run --output-format csv -- python -u tools/fhn_e2e.py 20 50 195325 > gpurun_out/fhn_e2e_b.txt 2>&1 || { echo "fhn e2e prof failed"; exit 1; }
