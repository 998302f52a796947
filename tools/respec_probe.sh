#!/bin/bash
# Burgers N=128 wall-clock under the re-speculation knobs (each step time-limited):
# NNGP_RESPEC_W (window), NNGP_RESPEC_PACKED (packed fits for the window), NNGP_RESPEC_PRIO (side
# stream at the least priority)
set -o pipefail
python -c "import torch, ctypes; h=ctypes.CDLL('libamdhip64.so'); lo=ctypes.c_int(); hi=ctypes.c_int(); h.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)); print('stream priority range least', lo.value, 'greatest', hi.value)"
for cfg in ${CONFIGS:-"W=4" "W=4 PACKED=1" "W=4 PRIO=1" "W=4 PACKED=1 PRIO=1" "W=2" "W=2 PACKED=1" "W=8 PACKED=1"}; do
  env_args=""
  for kv in $cfg; do env_args="$env_args NNGP_RESPEC_$kv"; done
  echo "== $cfg"
  env $env_args timeout -k 10 120 python -u tools/burgers_probe.py || exit $?
done
