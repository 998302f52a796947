#!/bin/bash
# Round 3, session Q: the parked-fit resume on the two-level kernel (4 / 2 waves per fit by the
# device-side parked count; an all-+inf simplex takes one whole iteration per wave and round):
# kernel tests against the oracle, the resume knobs, real FHN-PDE d=800 corrections and the
# d=800 N=512 run to convergence with the resume shapes off / default / forced.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_knobs.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "predict or knob" > $O/r3q_kernels.log 2>&1 &&
for cfg in "NNGP_RESUME_W4=0 NNGP_RESUME_W2=0" "NNGP_RESUME_W4=256" "NNGP_RESUME_W4=0 NNGP_RESUME_W2=0" "NNGP_RESUME_W4=256" "NNGP_NM_PARK=100"; do
  echo "== $cfg"; env $cfg timeout -k 10 120 python -u tools/fhn_fits_probe.py 4 || exit 1
  env $cfg timeout -k 10 120 python -u tools/fhn_e2e.py 20 50 195325 || exit 1
done > $O/r3q_resume.txt 2>&1 &&
for cfg in "NNGP_RESUME_W4=0 NNGP_RESUME_W2=0" "NNGP_RESUME_W4=256"; do
  echo "== $cfg"; env $cfg timeout -k 10 120 python -u tools/nm_probe.py park || exit 1
done > $O/r3q_park.txt 2>&1
rc=$?
tail -3 $O/r3q_kernels.log; grep -v amdgpu.ids $O/r3q_resume.txt | grep -E "==|slice|FHN|rows"; grep -v amdgpu.ids $O/r3q_park.txt
exit $rc
