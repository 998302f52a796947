#!/bin/bash
# Round 3, session C: halo-exchange latency (split-slice FHN-PDE question), 12 null-kernel windows
# under WRITE_SIZE (does the 344 KiB write appear without the fine kernel?), contracted-build K on
# Hopf / TomLab; before them the whole -m gpu suite (published-scale fixtures) and smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider --durations=20 > $O/r3c_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3c_smoke.log 2>&1 &&
timeout -k 5 60 scratch_bin/ubench_halo > $O/r3c_halo.txt 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/r3c_pmc_null -o run --output-format csv -- python3 tools/pmc_probe.py null 12 > $O/r3c_pmc_null.log 2>&1 &&
timeout -k 10 300 python -u tools/contract_k_probe.py > $O/r3c_contract_k.txt 2>&1
rc=$?
tail -25 $O/r3c_tests.log; tail -2 $O/r3c_smoke.log; cat $O/r3c_halo.txt $O/r3c_contract_k.txt
exit $rc
