#!/bin/bash
# r03: the mixed-scene shade (k_path_shade_full) at 5 / 6 waves per SIMD (RT_FULL_WAVES) against 4
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
V=$PWD/computational_ray_tracer_amd/lib/variants
SETS="cfg4:b0,f5,f6" ROUNDS=2 bash scripts/gpu_ab_sets.sh
