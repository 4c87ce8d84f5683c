#!/bin/bash
# r04 ab1 on one box: the GPU suite on the default build (all: compact 36-B BVH tiles + any-hit walks on the closest-hit
# BVH + coalesced radix scatter + 64-B NEE records), then interleaved bench A/Bs of
#   base  round-3 final build (ed6d035e)
#   all   rsc + the 64-B NEE records + lean mixed-scene camera samples
#   pk    all + the slab test in packed FMAs
#   gat   pk + the last ray-sort pass gathers the rays (the trace reads the sorted queue in order)
#   g4    gat + k_generate without pdf registers when lean (the default build); g5: the same at 5 waves/SIMD;
#   cs    g4 + incoherent shadow-ray waves compacted like closest-hit ones (single leaf)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab1_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r04ab1_t.log; [ $rc -ne 0 ] && exit $rc
export RTMI_AB_COMPAT=1
SETS="cfg4:base,g4,g4+RTMI_BVH_ANY=2/4 cornell:base,g4,cs cfg3:base,g4" ROUNDS=2 bash scripts/gpu_ab_sets.sh
