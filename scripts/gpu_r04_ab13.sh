#!/bin/bash
# r04 ab13: lane l starts its batch after lane l - 1's camera rays (RTMI_LANE_OFFSET=1) against both lanes at once
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RTMI_AB_COMPAT=1 SETS="cornell:lo,lo+RTMI_LANE_OFFSET=1 cfg3:lo,lo+RTMI_LANE_OFFSET=1 cfg4:lo,lo+RTMI_LANE_OFFSET=1" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
