#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
# A/B of the kernel variants in computational_ray_tracer_amd/lib/variants/*.so over bench configs:
#   CFGS="cornell cfg3 cfg4" [WITH_TESTS=1] bash scripts/gpu_ab_cfgs.sh
if [ -n "$WITH_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_tmp.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_tmp.log; [ $rc -ne 0 ] && exit $rc
fi
for c in ${CFGS:-cfg3 cfg4}; do
  s=${AB_STEPS:-2}; [ $c = cornell ] && s=${AB_STEPS_CORNELL:-6}
  echo "== $c"; BENCH_ARGS="--config $c" BENCH_STEPS=$s bash scripts/gpu_ab.sh || exit 1
done
