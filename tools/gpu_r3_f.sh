#!/bin/bash
# Round 3, session F: (1) Hopf group RHS with carried bank-masked registers (13 VALU per RHS
# instead of 16); (2) the likelihood evaluation without the pivot/diagonal selects, with the
# pivot's sqrt/reciprocal on their short sequences and the SE kernel's exp without the overflow
# path (scratch_bin/ub_{old,new}_M: same out hash, cycles per eval).  Per-step probes, the
# headline bench under rocprofv3 --kernel-trace --stats, the whole -m gpu suite, smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for M in 16 20 24; do for v in old new; do timeout -k 5 60 scratch_bin/ub_${v}_$M || exit 1; done; done > $O/r3f_gpeval.txt 2>&1 &&
timeout -k 10 180 python -u tools/lane_group_probe.py > $O/r3f_lane_group.txt 2>&1 &&
timeout -k 10 240 python -u tools/contract_probe.py > $O/r3f_contract_probe.txt 2>&1 &&
timeout -k 10 120 python -u tools/nm_probe.py > $O/r3f_nm_probe.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3f_bench -o run --output-format csv -- python3 bench.py --no-extras > $O/r3f_bench.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=10 > $O/r3f_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3f_smoke.log 2>&1
rc=$?
cat $O/r3f_gpeval.txt $O/r3f_lane_group.txt $O/r3f_contract_probe.txt $O/r3f_nm_probe.txt; grep -h '"metric"' $O/r3f_bench.log | cut -c1-400; tail -3 $O/r3f_tests.log; tail -1 $O/r3f_smoke.log
exit $rc
