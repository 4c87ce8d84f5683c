#!/bin/bash
# GPU-box check of a build: smoke, the -m gpu parity suite (stops on the first failure), then the multi-step bench
# lines of scripts/gpu_bench_cfgs.sh.   TAG=r03b [CONFIGS="cfg3 cfg4"] [PYTEST_K="expr"] bash scripts/gpu_test_bench.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -ne 0 ] && exit $rc
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
fi
[ -n "$NO_BENCH" ] && exit 0
TAG=$TAG bash scripts/gpu_bench_cfgs.sh
