#!/bin/bash
# r03: mixed-scene NEE at 5 waves per SIMD with a 20- / 16-entry any-hit stack (LDS then admits 5 blocks per CU)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/computational_ray_tracer_amd/lib/variants
RTMI_LIB=$V/n5s20.so RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cfg4 or nee" > gpurun_out/ab5_t.log 2>&1
rc=$?; echo "n5s20 tests rc=$rc"; tail -n 2 gpurun_out/ab5_t.log; [ $rc -ne 0 ] && exit $rc
SETS="cfg4:b0,n5s20,n5s16,s20" ROUNDS=2 bash scripts/gpu_ab_sets.sh
