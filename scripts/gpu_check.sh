#!/bin/bash
# GPU-box check: smoke, the -m gpu parity suite, a short bench.  Stops at the first crash/timeout.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "host cpus: $(nproc)"; lscpu | grep "Model name"
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-2} --warmup 1 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
