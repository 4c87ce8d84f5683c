#!/bin/bash
# GPU-box profiling: bench, rocprofv3 kernel-trace stats, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-4} --warmup 1 --cpu-seconds 10 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch_$TAG.log 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o pmc --output-format csv -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write_$TAG.log 2>&1
rc=$?; echo "rocprof write rc=$rc"; exit $rc
