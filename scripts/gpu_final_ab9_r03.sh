#!/bin/bash
# Final evidence of the committed build (r03zc, counters installed before the bench lines), then the CFG4
# runtime-option A/B (no material bins / three lanes).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=r03zc bash scripts/gpu_final_ab_r03.sh || exit 1
bash scripts/gpu_ab9_r03.sh
