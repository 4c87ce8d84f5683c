#!/bin/bash
# r04 ab7 on the final build (cur = its copy): batches in flight (lanes) x batch size, env only; the NEE sort in two
# 9-bit passes over a 6-bit-per-axis Morton key (nee9 + RTMI_SORT_NEE=1/6) against three 8-bit passes over 8 bits
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RTMI_AB_COMPAT=1 SETS="cornell:cur,cur+RTMI_LANES=4+RTMI_BATCH_SAMPLES=8388608,cur+RTMI_LANES=3+RTMI_BATCH_SAMPLES=8388608 cfg4:cur,nee9+RTMI_SORT_NEE=1/6,cur+RTMI_LANES=4+RTMI_BATCH_SAMPLES=8388608" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
