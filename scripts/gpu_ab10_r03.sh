#!/bin/bash
# r03: CFG4 ray-sort key origin-major (RTMI_SORT_BITS=3/3/1: the contiguous per-XCD shards then hold spatial regions)
# against the mixed-scene default direction-major; the sampler's PCG advance on the scalar unit when the wave shares
# the jump (RT_PCG_UNIFORM, k_generate)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RTMI_LIB=$PWD/computational_ray_tracer_amd/lib/variants/pcgu.so RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec \
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab10_t.log 2>&1
rc=$?; echo "pcgu tests rc=$rc"; tail -n 2 gpurun_out/ab10_t.log; [ $rc -ne 0 ] && exit $rc
SETS="cornell:b2,pcgu cfg4:b2,b2+RTMI_SORT_BITS=3/3/1" ROUNDS=3 bash scripts/gpu_ab_sets.sh
