#!/bin/bash
# contracted build + LinGrid check: bitwise RK suite, contracted tolerance suite, per-step probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_contract.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rk_ or contract or paged or group or field or rhs" > gpurun_out/ra_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/contract_probe.py > gpurun_out/contract_probe.txt 2>&1
rc=$?
tail -4 gpurun_out/ra_tests.log; cat gpurun_out/contract_probe.txt
exit $rc
