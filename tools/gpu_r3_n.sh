#!/bin/bash
# Round 3, session N: the rebuilt tree (container re-created) re-validated on MI355X: the whole
# -m gpu suite, smoke, the default bench line and a rocprofv3 kernel-trace summary of the
# headline bench and of the FHN-PDE d=800 N=512 run to convergence.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=10 > $O/r3n_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3n_smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/r3n_bench.json 2> $O/r3n_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3n_prof -o run --output-format csv -- python3 bench.py --no-extras > $O/r3n_prof_bench.json 2> $O/r3n_prof_bench.err &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r3n_fhn -o run --output-format csv -- python3 tools/fhn_e2e.py 20 50 195325 > $O/r3n_fhn_e2e.txt 2>&1
rc=$?
tail -3 $O/r3n_tests.log; tail -1 $O/r3n_smoke.log; cat $O/r3n_bench.json | cut -c1-600; tail -2 $O/r3n_bench.err; tail -3 $O/r3n_fhn_e2e.txt
exit $rc
