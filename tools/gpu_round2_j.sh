#!/bin/bash
# tail hand-off cap on real FHN-PDE d=800 corrections (after the failed-factorization early exit)
set -o pipefail
mkdir -p gpurun_out
for cap in 70 40 120 200 0; do
  echo "== NNGP_NM_PARK=$cap"
  NNGP_NM_PARK=$cap timeout -k 10 300 python -u tools/fhn_fits_probe.py 4 2>&1 | grep "slice" || exit 1
done
