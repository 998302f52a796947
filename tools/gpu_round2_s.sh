#!/bin/bash
# kNN select kernel time by training-set size (K = keys per thread) -- nngp_knn at d=128, m=15
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rs_knn -o run --output-format csv -- python3 tools/knn_probe.py > gpurun_out/rs_knn.log 2>&1 || { tail -20 gpurun_out/rs_knn.log; exit 1; }
grep -h "knn" $(find gpurun_out/rs_knn -name "*kernel_stats.csv") | cut -d, -f1-4
