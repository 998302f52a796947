#!/bin/bash
# Round 3, session H: the likelihood core with lane masks recomputed where used (no SGPR spill
# traffic), the failed-pivot state as a wave mask, no set-0 tail form at MAXM = 20 (new padded
# size 18 for m = 17, 18).  (1) ubench old/new (same out hash expected), (2) dynamic instruction
# counts of one evaluation (PMC), (3) correction timings, (4) FHN-PDE d=800 field kernel PMC
# (where a stage's cycles go; pair kernel with compile-time LDS images, both layouts), (5) FHN e2e, (6) the whole -m gpu suite and smoke.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for M in 16 18 20 24; do for v in old new; do timeout -k 5 60 scratch_bin/ub_${v}_$M | sed "s/^/$v /" || exit 1; done; done > $O/r3h_gpeval.txt 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d $O/r3h_pmc_ubold -o run --output-format csv -- scratch_bin/ub_old_20 > $O/r3h_pmc_ubold.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d $O/r3h_pmc_ubnew -o run --output-format csv -- scratch_bin/ub_new_20 > $O/r3h_pmc_ubnew.log 2>&1 &&
timeout -k 10 120 python -u tools/nm_probe.py > $O/r3h_nm_probe.txt 2>&1 &&
timeout -k 10 120 python -u tools/field_probe.py fhn > $O/r3h_field.txt 2>&1 &&
NNGP_FHN_PS=1024 timeout -k 10 120 python -u tools/field_probe.py fhn | sed "s/^/ps1024 /" >> $O/r3h_field.txt 2>&1 &&
NNGP_FHN_PAIR=0 timeout -k 10 120 python -u tools/field_probe.py fhn | sed "s/^/element /" >> $O/r3h_field.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d $O/r3h_pmc_fhnA -o run --output-format csv -- python3 tools/field_probe.py fhn > $O/r3h_pmc_fhnA.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $O/r3h_pmc_fhnB -o run --output-format csv -- python3 tools/field_probe.py fhn > $O/r3h_pmc_fhnB.log 2>&1 &&
timeout -k 10 120 python3 tools/fhn_e2e.py 20 50 195325 > $O/r3h_fhn_e2e.txt 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=10 > $O/r3h_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3h_smoke.log 2>&1
rc=$?
cat $O/r3h_gpeval.txt $O/r3h_nm_probe.txt $O/r3h_field.txt; grep -h FHN $O/r3h_fhn_e2e.txt; tail -3 $O/r3h_tests.log; tail -1 $O/r3h_smoke.log
exit $rc
