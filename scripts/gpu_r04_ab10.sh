#!/bin/bash
# r04 ab10: k_path_nee at 5 waves per SIMD (96 VGPRs + 104 B spill, any-hit stack 20) and the 20-entry any-hit stack
# alone, against the r04a final build (cur)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
RTMI_AB_COMPAT=1 SETS="cfg4:cur,nee5,as20 cfg3:cur,as20" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
exit 0
