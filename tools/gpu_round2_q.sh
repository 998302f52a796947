#!/bin/bash
# kernel stats of the Burgers N=128 run: unfused launch chain vs the fused chain
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
NNGP_CHAIN=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/rq_unfused -o run -- python3 tools/burgers_probe.py > gpurun_out/rq_unfused.log 2>&1 || { tail -20 gpurun_out/rq_unfused.log; exit 1; }
NNGP_CHAIN=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/rq_chain -o run -- python3 tools/burgers_probe.py > gpurun_out/rq_chain.log 2>&1 || { tail -20 gpurun_out/rq_chain.log; exit 1; }
grep early_stop gpurun_out/rq_unfused.log gpurun_out/rq_chain.log
for f in $(find gpurun_out/rq_unfused gpurun_out/rq_chain -name "*kernel_stats.csv"); do echo "== $f"; cut -d, -f1-4 $f | head -12; done
