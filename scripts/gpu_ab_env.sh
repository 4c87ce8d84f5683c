#!/bin/bash
# A/B of runtime options (environment variables) on one box, interleaved: VARIANTS="name:ENV=1,ENV2=0 ..."
# CONFIGS="cfg3 cfg4", ROUNDS=2.  One bench line per (round, variant, config).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    n=${v%%:*}; envs=$(echo ${v#*:} | tr ',' ' ')
    for c in ${CONFIGS:-cfg3 cfg4}; do
      steps=2; [ $c == cornell ] && steps=4
      env $envs timeout -k 10 300 python bench.py --config $c --steps $steps --warmup 1 --no-cpu-baseline \
        > gpurun_out/abenv_${n}_${c}_$r.log 2>&1 || { echo "$n $c failed"; tail -3 gpurun_out/abenv_${n}_${c}_$r.log; exit 1; }
      python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/abenv_${n}_${c}_$r.log') if x.startswith('{')][-1])
print('round $r', '$n', '$c', d['value'], d['stage_ms'])"
    done
  done
done
