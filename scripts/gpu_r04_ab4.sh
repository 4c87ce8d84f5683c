#!/bin/bash
# r04 ab4: the any-hit BVH's SAH parameters (0/4: the shadow rays on the closest-hit BVH itself) (RTMI_BVH_ANY="cost/leaf"; the CPU walk counts trade node visits for
# triangle tests) on the build with 64 bins and closest-hit node cost 2.5 (c25, the default build); Cornell against
# round 3; then where the Cornell kernels wait (SQ wait / LDS / SMEM counters).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bvh.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab4_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r04ab4_t.log; [ $rc -ne 0 ] && exit $rc
RTMI_AB_COMPAT=1 SETS="cfg4:c25,c25+RTMI_BVH_ANY=1.5/4,c25+RTMI_BVH_ANY=2/3,c25+RTMI_BVH_ANY=0/4 cfg3:c25,c25+RTMI_BVH_ANY=1.5/4,c25+RTMI_BVH_ANY=0/4 cornell:base,c25" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
# SIMD efficiency of the walks (RT_SIMD_STATS measurement build: lanes busy per node / triangle step)
for c in cfg3 cfg4; do
  RTMI_LIB=$PWD/computational_ray_tracer_amd/lib/variants/simd.so RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec RTMI_LANES=1 \
    timeout -k 10 300 python bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --project-shards 0 > gpurun_out/simd_r04_$c.log 2>&1
  rc=$?; echo "simd $c rc=$rc"; grep SIMD gpurun_out/simd_r04_$c.log | tail -2; [ $rc -ne 0 ] && exit $rc
done
CFG=cornell TAG=r04a bash scripts/gpu_pmc_cornell.sh || exit 1
exit 0
