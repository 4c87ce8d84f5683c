#!/bin/bash
# r04 ab9: closest-hit SAH node cost and leaf size again on the DP-collapsed build (cur = r04a final), env only
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RTMI_AB_COMPAT=1 SETS="cfg3:cur,cur+RTMI_BVH_CI=2,cur+RTMI_BVH_CI=3,cur+RTMI_BVH_LEAF=3 cfg4:cur,cur+RTMI_BVH_CI=2,cur+RTMI_BVH_CI=3,cur+RTMI_BVH_LEAF=3" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
