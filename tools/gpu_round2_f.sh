#!/bin/bash
# FHN-PDE d=800 N=512 to convergence under speculation policies (bound lifted; re-speculation window)
set -o pipefail
mkdir -p gpurun_out
for cfg in "NNGP_SPEC_MAX_FITS=0" "NNGP_SPEC_MAX_FITS=100000000 NNGP_RESPEC_W=0" "NNGP_SPEC_MAX_FITS=100000000 NNGP_RESPEC_W=1" "NNGP_SPEC_MAX_FITS=100000000 NNGP_RESPEC_W=4"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python -u tools/fhn_e2e.py 20 50 195325 2>&1 | grep "FHN-PDE" || exit 1
done
for cfg in "NNGP_SPEC_MAX_FITS=0" "NNGP_SPEC_MAX_FITS=100000000 NNGP_RESPEC_W=0"; do
  echo "== d=512 published config: $cfg"
  env $cfg timeout -k 10 200 python -u tools/fhn_e2e.py 16 25 195325 2>&1 | grep "FHN-PDE" || exit 1
done
