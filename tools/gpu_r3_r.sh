#!/bin/bash
# Round 3, session R: waves per all-+inf parked fit in the resume (NNGP_RESUME_INF_W = 1 / 2 / 4;
# with W > 1 such a fit takes W iterations per round): oracle tests with each, real FHN-PDE d=800
# corrections and the d=800 N=512 run to convergence.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for w in 2 4; do NNGP_RESUME_INF_W=$w timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "all_inf or fhn_pde_d800" || exit 1; done > $O/r3r_kernels.log 2>&1 &&
for w in 1 2 4 1 2 4; do
  echo "== INF_W=$w"; NNGP_RESUME_INF_W=$w timeout -k 10 120 python -u tools/fhn_fits_probe.py 4 || exit 1
  NNGP_RESUME_INF_W=$w timeout -k 10 120 python -u tools/fhn_e2e.py 20 50 195325 || exit 1
done > $O/r3r_resume.txt 2>&1
rc=$?
grep -E "passed|failed" $O/r3r_kernels.log; grep -E "==|slice|FHN-PDE" $O/r3r_resume.txt | grep -v "slice   1"
exit $rc
