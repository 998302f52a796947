#!/bin/bash
# Round 3, session C: halo-exchange latency (split-slice FHN-PDE question), 12 null-kernel windows
# under WRITE_SIZE (does the 344 KiB write appear without the fine kernel?), contracted-build K on
# Hopf / TomLab, and the bench (default flags) once.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 5 60 scratch_bin/ubench_halo > $O/r3c_halo.txt 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/r3c_pmc_null -o run --output-format csv -- python3 tools/pmc_probe.py null 12 > $O/r3c_pmc_null.log 2>&1 &&
timeout -k 10 400 python -u tools/contract_k_probe.py > $O/r3c_contract_k.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/r3c_fhn -o run --output-format csv -- python3 tools/fhn_e2e.py 20 50 195325 > $O/r3c_fhn_e2e.txt 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/r3c_bench.json 2> $O/r3c_bench.err
rc=$?
cat $O/r3c_halo.txt $O/r3c_contract_k.txt; tail -5 $O/r3c_bench.err; tail -c 3000 $O/r3c_bench.json
exit $rc
