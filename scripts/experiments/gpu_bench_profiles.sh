#!/bin/bash
# Bench lines + rocprofv3 kernel stats for C2 (default) and C3: gpurun_out/{bench,prof}_*.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o c2 --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c2_prof.log 2>&1 || exit 1
timeout -k 10 900 python bench.py --workload c3 --steps 5 --warmup 1 > gpurun_out/bench_c3.log 2>&1 || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o c3 --output-format csv -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_prof.log 2>&1 || exit 1
