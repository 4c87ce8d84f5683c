#!/bin/bash
# r03: three breadth-first BVH levels (1 + 8 + 64 nodes, 5.8 KB) staged in LDS instead of two (RT_BVH_TOP_LEVELS=3)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/computational_ray_tracer_amd/lib/variants
export RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec
RTMI_LIB=$V/top3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab8_t.log 2>&1
rc=$?; echo "top3 tests rc=$rc"; tail -n 2 gpurun_out/ab8_t.log; [ $rc -ne 0 ] && exit $rc
SETS="cfg3:b1,top3 cfg4:b1,top3" ROUNDS=3 bash scripts/gpu_ab_sets.sh
