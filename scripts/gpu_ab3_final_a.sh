#!/bin/bash
# r03: Cornell A/B of the pair append with and without the slot/hit prefetch, then the final-build evidence part a.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/computational_ray_tracer_amd/lib/variants
RTMI_LIB=$V/cpasp.so RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "cornell or concurrent or shards or cfg0 or sensor" > gpurun_out/ab3_t_cpasp.log 2>&1
rc=$?; echo "cpasp tests rc=$rc"; tail -n 2 gpurun_out/ab3_t_cpasp.log; [ $rc -ne 0 ] && exit $rc
SETS="cornell:cpa,cpasp" ROUNDS=3 bash scripts/gpu_ab_sets.sh || exit 1
TAG=r03za PART=a bash scripts/gpu_final_r03.sh
