#!/bin/bash
# overlapped batch: fits per row of the packed kernel's work queues (order of query completion)
set -o pipefail
for r in 8 1 2 4 8 2; do echo "== NNGP_NM_REFILL=$r"; NNGP_NM_REFILL=$r timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep "early_stop=None" || exit 1; done
