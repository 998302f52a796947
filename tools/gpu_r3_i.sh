#!/bin/bash
# Round 3, session I: the likelihood core with the row scalars (L_jj, 1/L_jj, z, alpha) in LDS
# slots written by every lane of the row (no owner selects), and 3-address fma for the exp's Horner
# steps (fma3: the library and ub_f3 carry it); the FHN pair kernel with the next stage's partial
# sums formed while the neighbour reads are in flight and the step update accumulated per stage: ubench old (HEAD) / new / fma3 with hashes,
# dynamic counts (PMC), correction timings, FHN e2e, Burgers to convergence, whole -m gpu, smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
{ for M in 16 18 20 24; do for v in old new; do timeout -k 5 60 scratch_bin/ub_${v}_$M | sed "s/^/$v /" || exit 1; done; done;
  for M in 16 20; do timeout -k 5 60 scratch_bin/ub_f3_$M | sed "s/^/fma3 /" || exit 1; done; } > $O/r3i_gpeval.txt 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/r3i_pmc_ubnew -o run --output-format csv -- scratch_bin/ub_new_20 > $O/r3i_pmc_ubnew.log 2>&1 &&
timeout -k 10 120 python -u tools/nm_probe.py > $O/r3i_nm_probe.txt 2>&1 &&
timeout -k 10 120 python -u tools/field_probe.py fhn > $O/r3i_field.txt 2>&1 &&
timeout -k 10 120 python3 tools/fhn_e2e.py 20 50 195325 > $O/r3i_fhn_e2e.txt 2>&1 &&
timeout -k 10 120 python3 tools/burgers_probe.py > $O/r3i_burgers.txt 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=10 > $O/r3i_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3i_smoke.log 2>&1
rc=$?
cat $O/r3i_gpeval.txt $O/r3i_nm_probe.txt $O/r3i_field.txt; grep -h FHN $O/r3i_fhn_e2e.txt; tail -4 $O/r3i_burgers.txt; tail -3 $O/r3i_tests.log; tail -1 $O/r3i_smoke.log
exit $rc
