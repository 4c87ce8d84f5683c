#!/bin/bash
# r04 ab5: the DP-optimal 8-wide collapse (default build) against the greedy collapse (c25); the any-hit BVH at
# cost 1.5 on the DP build; CFG3 through the general (deferred, sorted NEE) kernels; Cornell with round 3's
# single generate kernel (genold) for the 0.6 % it lost.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab5_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r04ab5_t.log; [ $rc -ne 0 ] && exit $rc
RTMI_AB_COMPAT=1 SETS="cfg3:c25,dp,dp+RTMI_BVH_ANY=1.5/4,dp+RTMI_FULL_PATH=1 cfg4:c25,dp,dp+RTMI_BVH_ANY=1.5/4 cornell:dp,genold,dp+RTMI_FULL_PATH=1" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
