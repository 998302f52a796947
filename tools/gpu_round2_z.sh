#!/bin/bash
# overlapped batch stream priority (and the re-speculation stream's) on Burgers N=128
set -o pipefail
for bp in 0 1 0 1; do for rp in 0 1; do echo "== NNGP_BATCH_PRIO=$bp NNGP_RESPEC_PRIO=$rp"; NNGP_BATCH_PRIO=$bp NNGP_RESPEC_PRIO=$rp timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep "early_stop=None" || exit 1; done; done
