#!/bin/bash
# Round 3, session T: the park cap with the device-shaped resume (NNGP_NM_PARK 60 / 70 / 80 / 90),
# real FHN-PDE d=800 corrections and the d=800 N=512 run to convergence, twice each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for cap in 60 70 80 90 60 70 80 90; do
  echo "== PARK=$cap"; NNGP_NM_PARK=$cap timeout -k 10 120 python -u tools/fhn_fits_probe.py 4 || exit 1
  NNGP_NM_PARK=$cap timeout -k 10 120 python -u tools/fhn_e2e.py 20 50 195325 || exit 1
done > $O/r3t_park.txt 2>&1
rc=$?
grep -E "==|slice|FHN-PDE" $O/r3t_park.txt | grep -v "slice   1"
exit $rc
