#!/bin/bash
# Round 3, session B: (1) the GP-evaluation micro-benchmark, old layout vs pinned/shrunk-image
# layout, MAXM 16/20/24 (identical output hashes expected); (2) the GPU suite without the 110 s
# published Burgers Parareal run; (3) nnGP correction timings; (4) the fused chain under rocprofv3
# again (ordinary launch now); (5) PMC attribution passes of the fine kernel (FETCH / WRITE).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
{ for M in 16 20 24; do for v in old new; do timeout -k 5 60 scratch_bin/ub_${v}_$M | sed "s/^/$v /" || exit 1; done; done; } > $O/r3b_ubench.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "not burgers_published_schedule_parareal" --durations=15 > $O/r3b_tests.log 2>&1 &&
timeout -k 10 120 python -u tools/nm_probe.py > $O/r3b_nm_probe.txt 2>&1 &&
NNGP_NM_SPEC=1 timeout -k 10 120 python -u tools/nm_probe.py sweep > $O/r3b_nm_sweep_spec.txt 2>&1 &&
NNGP_NM_SPEC=0 timeout -k 10 120 python -u tools/nm_probe.py sweep > $O/r3b_nm_sweep_packed.txt 2>&1 &&
timeout -k 10 200 python -u tools/contract_probe.py > $O/r3b_contract_probe.txt 2>&1 &&
NNGP_CHAIN=1 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/r3b_chain -o run -- python3 tools/burgers_probe.py > $O/r3b_chain.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/r3b_pmc_write -o run --output-format csv -- python3 tools/pmc_probe.py > $O/r3b_pmc_write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/r3b_pmc_fetch -o run --output-format csv -- python3 tools/pmc_probe.py > $O/r3b_pmc_fetch.log 2>&1 &&
python3 tools/pmc_traffic.py $(find $O/r3b_pmc_fetch -name "*counter_collection.csv" | head -1) $(find $O/r3b_pmc_write -name "*counter_collection.csv" | head -1) $O/r3b_fine_kernel_traffic.json rk_group_kernel > $O/r3b_pmc_summary.txt 2>&1
rc=$?
cat $O/r3b_ubench.txt; tail -20 $O/r3b_tests.log; cat $O/r3b_nm_probe.txt $O/r3b_contract_probe.txt; tail -3 $O/r3b_chain.log; tail -3 $O/r3b_pmc_fetch.log
exit $rc
