#!/bin/bash
# One GPU session: bench (default), rocprofv3 kernel-trace stats of the bench's fine sweep and of the
# nnGP correction probe, PMC traffic passes.  Usage (via gpurun): bash tools/gpu_bench_profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed rc=$?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python bench.py --no-extras > $OUT/prof_bench_$TAG.json 2> $OUT/prof_bench_$TAG.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_bench_$TAG.err; exit 1; }
cat $OUT/prof_bench_$TAG.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_nm_$TAG -o run --output-format csv -- python tools/nm_probe.py > $OUT/nm_probe_$TAG.txt 2>&1 || { echo "rocprof nm failed"; tail -5 $OUT/nm_probe_$TAG.txt; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_burgers_$TAG -o run --output-format csv -- python tools/burgers_probe.py > $OUT/burgers_probe_$TAG.txt 2>&1 || { echo "rocprof burgers failed"; tail -5 $OUT/burgers_probe_$TAG.txt; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_gp_$TAG -o run --output-format csv -- python tools/gp_probe.py > $OUT/gp_probe_$TAG.txt 2>&1 || { echo "rocprof gp failed"; tail -5 $OUT/gp_probe_$TAG.txt; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$TAG -o run --output-format csv -- python bench.py --no-extras --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_fetch_$TAG.err || { echo "pmc fetch failed"; tail -5 $OUT/pmc_fetch_$TAG.err; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$TAG -o run --output-format csv -- python bench.py --no-extras --steps 2 --warmup 0 > /dev/null 2> $OUT/pmc_write_$TAG.err || { echo "pmc write failed"; tail -5 $OUT/pmc_write_$TAG.err; exit 1; }
python tools/pmc_traffic.py $(find $OUT/pmc_fetch_$TAG -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write_$TAG -name "*counter_collection.csv" | head -1) $OUT/fine_kernel_traffic_$TAG.json rk_group_kernel || { echo "pmc parse failed"; exit 1; }
find $OUT/prof_$TAG $OUT/prof_nm_$TAG $OUT/prof_burgers_$TAG $OUT/prof_gp_$TAG $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG -name "*.csv" | head -20
