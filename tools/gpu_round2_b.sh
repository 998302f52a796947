#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/respec_probe.sh > gpurun_out/respec_probe.txt 2>&1 || { echo "respec probe failed"; tail -20 gpurun_out/respec_probe.txt; exit 1; }
grep -v "^W20\|^E20" gpurun_out/respec_probe.txt
bash tools/gpu_published.sh
