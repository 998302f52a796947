#!/bin/bash
# Round 3, session G (re-entry after a container rebuild): the current tree's whole -m gpu suite,
# smoke, the default bench line, and the headline bench under rocprofv3 --kernel-trace --stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=10 > $O/r3g_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3g_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/r3g_bench.json 2> $O/r3g_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3g_prof -o run --output-format csv -- python3 bench.py --no-extras > $O/r3g_prof.log 2>&1
rc=$?
tail -3 $O/r3g_tests.log; tail -1 $O/r3g_smoke.log; tail -c 600 $O/r3g_bench.json; grep -h '"metric"' $O/r3g_prof.log | cut -c1-300
exit $rc
