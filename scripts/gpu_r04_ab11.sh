#!/bin/bash
# r04 ab11: bench step size (sample indices per step: 16 = 2 batches of 8 on the two lanes, 32 = 4 batches, 48 = 6)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for c in cornell cfg3; do
    for k in 16 32 48; do
      s=6; [ $c = cfg3 ] && s=3
      timeout -k 10 300 python bench.py --config $c --steps $s --warmup 1 --spp-per-step $k --no-cpu-baseline --project-shards 0 > gpurun_out/ab11_${c}_${k}_$r.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "$c $k rc=$rc"; tail -3 gpurun_out/ab11_${c}_${k}_$r.log; exit $rc; }
      python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/ab11_${c}_${k}_$r.log') if x.startswith('{')][-1])
print('round $r', '$c', 'spp/step $k', d['value'], d['ms_per_step'])"
    done
  done
done
exit 0
