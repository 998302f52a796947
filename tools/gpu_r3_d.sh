#!/bin/bash
# Round 3, session D: kernel trace of the FHN-PDE d=800 N=512 run to convergence, then the bench
# (default flags) once.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r3d_fhn -o run --output-format csv -- python3 tools/fhn_e2e.py 20 50 195325 > $O/r3d_fhn_e2e.txt 2>&1 &&
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $O/r3d_burg -o run -- python3 tools/burgers_probe.py > $O/r3d_burg.txt 2>&1 &&
for cap in 50 100 140; do NNGP_NM_PARK=$cap timeout -k 10 120 python3 tools/fhn_e2e.py 20 50 195325 | sed "s/^/park=$cap /" || exit 1; done > $O/r3d_park_sweep.txt 2>&1 &&
timeout -k 10 800 python -u bench.py > $O/r3d_bench.json 2> $O/r3d_bench.err
rc=$?
grep FHN $O/r3d_fhn_e2e.txt; grep FHN $O/r3d_park_sweep.txt; tail -5 $O/r3d_bench.err; tail -c 3000 $O/r3d_bench.json
exit $rc
