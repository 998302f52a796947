#!/bin/bash
# Round 3, first GPU session: the whole -m gpu suite (new published-scale, 8-rank and knob tests),
# smoke, then the fused chain under rocprofv3 once more (the round-2 exit-time SIGSEGV), with the
# process's mappings dumped at exit.  Each GPU step time-limited, chained with &&.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations=25 > gpurun_out/r3a_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3a_smoke.log 2>&1 &&
NNGP_CHAIN=1 NNGP_PROBE_MAPS=gpurun_out/r3a_chain_maps.txt timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a_chain -o run -- python3 tools/burgers_probe.py > gpurun_out/r3a_chain.log 2>&1
rc=$?
tail -30 gpurun_out/r3a_tests.log; tail -3 gpurun_out/r3a_smoke.log 2>/dev/null; tail -5 gpurun_out/r3a_chain.log 2>/dev/null
exit $rc
