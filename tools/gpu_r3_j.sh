#!/bin/bash
# Round 3, session J: the likelihood core with the forward solve fused into the Cholesky columns
# (z_j from column j's L_jj / RN(1/L_jj) in registers), L_jj / RN(1/L_jj) / z in LDS scalar slots
# for the back solve (no owner selects but alpha's), 3-address fma in the exp's Horner steps
# (ub_old = HEAD's core with the fma3 math, ub_new = this); the FHN pair kernel with the next
# stage's partial sums in source order before the stencil (no pin) and the step update per stage;
# the ThomasLabyrinth sine without its non-finite select (NaN arises on its own).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for M in 16 18 20 24; do for v in old new; do timeout -k 5 60 scratch_bin/ub_${v}_$M | sed "s/^/$v /" || exit 1; done; done > $O/r3j_gpeval.txt 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/r3j_pmc_ubnew -o run --output-format csv -- scratch_bin/ub_new_20 > $O/r3j_pmc_ubnew.log 2>&1 &&
timeout -k 10 120 python -u tools/nm_probe.py > $O/r3j_nm_probe.txt 2>&1 &&
timeout -k 10 120 python -u tools/field_probe.py fhn > $O/r3j_field.txt 2>&1 &&
timeout -k 10 180 python -u tools/lane_group_probe.py > $O/r3j_lane_group.txt 2>&1 &&
timeout -k 10 240 python -u tools/contract_probe.py > $O/r3j_contract_probe.txt 2>&1 &&
timeout -k 10 120 python3 tools/fhn_e2e.py 20 50 195325 > $O/r3j_fhn_e2e.txt 2>&1 &&
timeout -k 10 120 python3 tools/burgers_probe.py > $O/r3j_burgers.txt 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider --durations=10 > $O/r3j_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r3j_smoke.log 2>&1
rc=$?
cat $O/r3j_gpeval.txt $O/r3j_nm_probe.txt $O/r3j_field.txt $O/r3j_lane_group.txt $O/r3j_contract_probe.txt; grep -h FHN $O/r3j_fhn_e2e.txt; tail -4 $O/r3j_burgers.txt; tail -3 $O/r3j_tests.log; tail -1 $O/r3j_smoke.log
exit $rc
