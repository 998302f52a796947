#!/bin/bash
# FHN-PDE d=800 N=512 end-to-end kernel profile + published-scale nnGP seed spread
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fhn_e2e -o run --output-format csv -- python -u tools/fhn_e2e.py 20 50 195325 > gpurun_out/fhn_e2e.txt 2>&1 || { echo "fhn e2e failed"; tail -20 gpurun_out/fhn_e2e.txt; exit 1; }
grep -v "^W20\|^E20" gpurun_out/fhn_e2e.txt | tail -3
NNGP_PUBLISHED=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_published.py -m gpu -v -s --timeout 600 --timeout-method thread -k "nngp" > gpurun_out/published_nngp.log 2>&1
rc=$?
grep -E "published|passed|failed" gpurun_out/published_nngp.log | tail -8
exit $rc
