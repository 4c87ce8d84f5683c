#!/bin/bash
# GPU: parity suite, then short benches of the selected configs (default: cornell cfg3 cfg4), one line each.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-all}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS:-cornell cfg3 cfg4}; do
  steps=4; [ $c != cornell ] && steps=2
  timeout -k 10 400 python bench.py --config $c --steps $steps --warmup 1 --no-cpu-baseline > gpurun_out/bench_${c}_$TAG.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$c rc=$rc"; tail -5 gpurun_out/bench_${c}_$TAG.log; exit $rc; }
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/bench_${c}_$TAG.log') if x.startswith('{')][-1])
r=d['roofline']
print('$c', d['value'], d['stage_ms'], r['kernel'], r['avg_launch_ms'], r['frac'], r.get('valu',{}).get('frac'))"
done
