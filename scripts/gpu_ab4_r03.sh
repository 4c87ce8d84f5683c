#!/bin/bash
# r03: static chunks of 2 / 3 / 4 items per thread on the single-leaf path (one parked block append per chunk), then
# the >= 8-step bench lines of the committed default build (gpu_final_r03.sh PART=b).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/computational_ray_tracer_amd/lib/variants
for v in si4 si3; do
RTMI_LIB=$V/$v.so RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec timeout -k 10 600 \
  python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab4_t_$v.log 2>&1
rc=$?; echo "$v tests rc=$rc"; tail -n 2 gpurun_out/ab4_t_$v.log; [ $rc -ne 0 ] && exit $rc
done
SETS="cornell:si2,si3,si4" ROUNDS=3 bash scripts/gpu_ab_sets.sh || exit 1
TAG=r03za PART=b bash scripts/gpu_final_r03.sh
