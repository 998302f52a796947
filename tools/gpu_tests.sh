#!/bin/bash
# GPU parity suite + smoke on the box; each GPU step time-limited, chained with &&.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log; tail -3 gpurun_out/smoke.log 2>/dev/null
exit $rc
