#!/bin/bash
# Quick GPU perf probe: path-mode bench (no CPU baseline) + the GPU parity suite, stage times only.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-4} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/quick.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ -n "$WITH_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
fi
python3 - <<'PY'
import json
l=[x for x in open('gpurun_out/quick.log') if x.startswith('{')][-1]
d=json.loads(l)
print('VALUE', d['value'], 'ms/step', d['ms_per_step'], d['stage_ms'], 'roofline', d['roofline']['frac'])
PY
