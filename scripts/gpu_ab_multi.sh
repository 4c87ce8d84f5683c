#!/bin/bash
# One GPU call, several experiments: kernel variants (lib/variants/*.so) on CFGS, then runtime-option variants
# (ENV_VARIANTS="name:ENV=1,...") on ENV_CONFIGS with the default library.  Stops at the first failure.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
if [ -n "$CFGS" ]; then CFGS="$CFGS" bash scripts/gpu_ab_cfgs.sh || exit 1; fi
if [ -n "$ENV_VARIANTS" ]; then VARIANTS="$ENV_VARIANTS" CONFIGS="${ENV_CONFIGS:-cornell}" bash scripts/gpu_ab_env.sh || exit 1; fi
exit 0
