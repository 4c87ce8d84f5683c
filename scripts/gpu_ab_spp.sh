#!/bin/bash
# A/B of (environment, bench arguments) pairs on one box, interleaved: one bench line per (round, variant).
# VARIANTS="name|ENV=1,ENV2=2|--spp-per-step 16 ..." (fields separated by '|'; ROUNDS=2, CONFIG=cornell)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    IFS='|' read -r n envs args <<< "$v"
    envs=$(echo $envs | tr ',' ' '); args=$(echo $args | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --config ${CONFIG:-cornell} --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline $args \
      > gpurun_out/abspp_${n}_$r.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abspp_${n}_$r.log; exit 1; }
    python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/abspp_${n}_$r.log') if x.startswith('{')][-1])
print('round $r', '$n', d['value'], d['ms_per_step'], d['stage_ms'])"
  done
done
