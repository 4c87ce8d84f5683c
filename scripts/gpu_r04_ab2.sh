#!/bin/bash
# r04 ab2 on one box: the GPU suite on the default build, then interleaved bench A/Bs and single-lane kernel traces.
#   base  round-3 final build (ed6d035e)
#   def   the default build: 36-B tiles + separate any-hit BVH, 64-B NEE records, lean mixed-scene camera samples,
#         packed-FMA slab test, LDS-staged radix scatter (the trace gathers the sorted rays), last-depth emitter filter
#   rso   def with round 3's radix scatter (tiles of one item per thread)
#   def+RTMI_EMIT_FILTER=0: def tracing every ray at the last depth
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab2_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/r04ab2_t.log; [ $rc -ne 0 ] && exit $rc
export RTMI_AB_COMPAT=1
SETS="cfg4:base,def,rso,def+RTMI_EMIT_FILTER=0 cfg3:base,def,rso cornell:base,def" ROUNDS=2 bash scripts/gpu_ab_sets.sh || exit 1
unset RTMI_AB_COMPAT
for c in cfg4 cfg3; do
  RTMI_LANES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_r04b_$c -o kt --output-format csv -- \
    python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --project-shards 0 > gpurun_out/kt_r04b_$c.log 2>&1
  rc=$?; echo "kt $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
