#!/bin/bash
# Multi-step bench lines (>= 8 timed steps, 2 warmup) of the BASELINE configs on one GPU, one run each:
#   TAG=r03a CONFIGS="cornell cfg3 cfg4 cfg5" bash scripts/gpu_bench_cfgs.sh
# Lines land in gpurun_out/bench_<config>_<TAG>.log; stops at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03}
STEPS=${STEPS:-8}
mkdir -p gpurun_out
for c in ${CONFIGS:-cornell cfg3 cfg4 cfg5}; do
  timeout -k 10 400 python -u bench.py --config $c --steps $STEPS --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_${c}_$TAG.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$c rc=$rc"; tail -5 gpurun_out/bench_${c}_$TAG.log; exit $rc; }
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/bench_${c}_$TAG.log') if x.startswith('{')][-1])
print('$c', d['value'], d['ms_per_step'], d['stage_ms'])"
done
exit 0
