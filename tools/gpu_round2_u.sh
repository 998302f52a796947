#!/bin/bash
# fits kernels register-allocated for 3 waves per SIMD (MAXM <= 16): parity, then timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parareal.py -m gpu -x -q --timeout 300 --timeout-method thread -k "predict or nm or speculative or bitwise" > gpurun_out/ru_tests.log 2>&1 || { tail -40 gpurun_out/ru_tests.log; exit 1; }
tail -1 gpurun_out/ru_tests.log
timeout -k 10 200 python -u tools/nm_probe.py 2>&1 | grep "ms/correction" || exit 1
for i in 1 2; do timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep "early_stop=None" || exit 1; done
