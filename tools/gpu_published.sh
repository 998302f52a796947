#!/bin/bash
# published-scale K parity (tests/test_gpu_published.py): minutes of GPU time
set -o pipefail
mkdir -p gpurun_out
NNGP_PUBLISHED=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_published.py -m gpu -v -s --timeout 600 --timeout-method thread > gpurun_out/published.log 2>&1
rc=$?
grep -E "published|PASS|FAIL|passed|failed" gpurun_out/published.log | tail -12
exit $rc
