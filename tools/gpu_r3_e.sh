#!/bin/bash
# Round 3, session E: Burgers N=128 to convergence with the overlapped batch's stream kept off R CUs
# (NNGP_BATCH_CU_RESERVE), the run on a non-default stream (a CU-masked stream is a blocking one).
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
{ for R in 0 16 32 64; do for S in 0 1; do
    echo "== reserve=$R stream=$S"; NNGP_BATCH_CU_RESERVE=$R NNGP_PROBE_STREAM=$S timeout -k 10 120 python3 tools/burgers_probe.py || exit 1
  done; done; } > $O/r3e_reserve.txt 2>&1
rc=$?
grep -E "==|early_stop=None" $O/r3e_reserve.txt
exit $rc
