#!/bin/bash
# Round-3 evidence of the final build, in two GPU calls (PART=a / PART=b); stops at the first failure.
#   a: smoke, the -m gpu suite, single-lane kernel traces + PMC counters of Cornell / CFG3 / CFG4 (gpu_counters.sh)
#   b: >= 8-step bench lines of every BASELINE config (the default line with the CPU baseline)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-r03za}
if [ "${PART:-a}" = a ]; then
  timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_$TAG.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
  TAG=$TAG CONFIGS="${CONFIGS:-cornell cfg3 cfg4}" bash scripts/gpu_counters.sh || exit 1
else
  timeout -k 10 600 python -u bench.py --steps 8 --warmup 2 --cpu-seconds 10 > gpurun_out/bench_default_$TAG.log 2>&1
  rc=$?; echo "default bench rc=$rc"; tail -n 1 gpurun_out/bench_default_$TAG.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
  TAG=$TAG STEPS=8 CONFIGS="${CONFIGS:-cornell cfg3 cfg4 cfg5}" bash scripts/gpu_bench_cfgs.sh || exit 1
fi
exit 0
