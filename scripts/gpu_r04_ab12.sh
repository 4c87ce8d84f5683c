#!/bin/bash
# r04 ab12: lanes 1.. released from the pass-start join (lj = the default build after it) against the join
# (RTMI_LANE_JOIN=1, the round-4 behaviour); the -m gpu suite first (film order across lanes and passes)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab12_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r04ab12_t.log; [ $rc -ne 0 ] && exit $rc
RTMI_AB_COMPAT=1 SETS="cornell:lj+RTMI_LANE_JOIN=1,lj cfg3:lj+RTMI_LANE_JOIN=1,lj cfg4:lj+RTMI_LANE_JOIN=1,lj" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
