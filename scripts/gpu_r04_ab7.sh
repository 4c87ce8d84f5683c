#!/bin/bash
# r04 ab7: batches in flight (lanes) x batch size on the final build (cur = its copy), env only
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RTMI_AB_COMPAT=1 SETS="cornell:cur,cur+RTMI_LANES=4+RTMI_BATCH_SAMPLES=8388608,cur+RTMI_LANES=3+RTMI_BATCH_SAMPLES=8388608 cfg3:cur,cur+RTMI_LANES=4+RTMI_BATCH_SAMPLES=8388608" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
