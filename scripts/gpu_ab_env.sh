#!/bin/bash
# A/B of runtime settings: CASES="name:VAR=v,VAR2=w name2:..." (interleaved rounds, one process each).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for round in 1 2; do
  for cs in $CASES; do
    n=${cs%%:*}; envs=$(echo ${cs#*:} | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abe_$n.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -3 gpurun_out/abe_$n.log; exit $rc; }
    python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/abe_$n.log') if x.startswith('{')][-1])
print('round $round', '$n', d['value'], d['stage_ms'])"
  done
done
