#!/bin/bash
# re-speculation window width on Burgers N=128 after the select changes
set -o pipefail
for w in 4 1 2 3 4 2; do echo "== NNGP_RESPEC_W=$w"; NNGP_RESPEC_W=$w timeout -k 10 120 python -u tools/burgers_probe.py 2>&1 | grep "early_stop=None" || exit 1; done
