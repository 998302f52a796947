#!/bin/bash
# wave-per-pair D2 (d > 128): parity tests, then one correction's time with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parareal.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread -k "knn or predict or speculative or fhn or distributed or bitwise" > gpurun_out/rt_tests.log 2>&1 || { tail -40 gpurun_out/rt_tests.log; exit 1; }
tail -1 gpurun_out/rt_tests.log
for w in 0 1; do echo "== NNGP_D2_WAVES=$w"; NNGP_D2_WAVES=$w timeout -k 10 200 python -u tools/nm_probe.py 2>&1 | grep "ms/correction" || exit 1; done
