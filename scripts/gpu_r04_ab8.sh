#!/bin/bash
# r04 ab8: the simple path's primitive id in hitB.w (pk = the default build after it) against the r04a final build (cur)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab8_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r04ab8_t.log; [ $rc -ne 0 ] && exit $rc
RTMI_AB_COMPAT=1 SETS="cornell:cur,pk cfg3:cur,pk" ROUNDS=3 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
