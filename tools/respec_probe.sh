#!/bin/bash
# Burgers N=128 wall-clock for re-speculation windows (each step time-limited)
set -o pipefail
for w in ${WINDOWS:-0 2 4 8}; do
  echo "NNGP_RESPEC_W=$w"
  NNGP_RESPEC_W=$w timeout -k 10 120 python -u tools/burgers_probe.py || exit $?
done
