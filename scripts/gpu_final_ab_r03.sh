#!/bin/bash
# Final round-3 evidence of the committed build in one call: smoke, -m gpu, counters + single-lane traces (part a),
# which are then installed as profiles/counters_<config>.json on the box so that the >= 8-step bench lines of part b
# carry the PMC traffic / VALU of the same build.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-r03zb}
TAG=$T PART=a bash scripts/gpu_final_r03.sh || exit 1
for c in cornell cfg3 cfg4; do cp gpurun_out/cnt_${c}_$T.counters.json profiles/counters_$c.json || exit 1; done
TAG=$T PART=b bash scripts/gpu_final_r03.sh
