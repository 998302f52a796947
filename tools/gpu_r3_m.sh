#!/bin/bash
# Round 3, session M: the two-level speculative Nelder-Mead kernel (nm_spec2_kernel, 2 or 4 waves
# per fit for few fits; rows form their own candidates, the consume scan is one ballot): kernel tests against the oracle, correction timings with it off / auto /
# forced, the whole -m gpu suite and smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "predict" > $O/r3m_kernels.log 2>&1 &&
for v in 0 1 4; do NNGP_NM_LEVEL2=$v timeout -k 10 120 python -u tools/nm_probe.py level2 | sed "s/^/L$v /" || exit 1; done > $O/r3m_level2.txt 2>&1 &&
timeout -k 10 120 python -u tools/nm_probe.py > $O/r3m_nm_probe.txt 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=10 > $O/r3m_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3m_smoke.log 2>&1
rc=$?
tail -3 $O/r3m_kernels.log; grep -v amdgpu.ids $O/r3m_level2.txt; cat $O/r3m_nm_probe.txt; tail -3 $O/r3m_tests.log; tail -1 $O/r3m_smoke.log
exit $rc
