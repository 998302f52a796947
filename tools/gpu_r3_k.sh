#!/bin/bash
# Round 3, session K: the default bench line (all extras) on the committed tree, the headline bench
# under rocprofv3 --kernel-trace --stats, and the FHN-PDE d=800 N=512 run to convergence under the
# kernel trace (per-kernel shares of the correction and the fine sweep).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u bench.py > $O/r3k_bench.json 2> $O/r3k_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3k_prof -o run --output-format csv -- python3 bench.py --no-extras > $O/r3k_prof.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r3k_fhn -o run --output-format csv -- python3 tools/fhn_e2e.py 20 50 195325 > $O/r3k_fhn_e2e.txt 2>&1
rc=$?
tail -c 700 $O/r3k_bench.json; grep -h '"metric"' $O/r3k_prof.log | cut -c1-300; grep FHN $O/r3k_fhn_e2e.txt
exit $rc
