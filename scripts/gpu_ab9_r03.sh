#!/bin/bash
# r03: CFG4 runtime options against the default: one mixed shade kernel without material bins, three lanes
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
SETS="cfg4:b1,b1+RTMI_MAT_BINS=0,b1+RTMI_LANES=3" ROUNDS=2 bash scripts/gpu_ab_sets.sh
