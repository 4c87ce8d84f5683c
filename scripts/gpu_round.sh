#!/bin/bash
# GPU-box round check: smoke, the -m gpu parity suite, the default bench line (with CPU baseline), short
# cfg3/cfg4 bench lines, and a single-lane (RTMI_LANES=1) rocprofv3 kernel trace of the default bench, whose
# per-kernel durations are not shared with a concurrent lane.  Stops at the first failure; every GPU step runs
# under its own time limit.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r02}
mkdir -p gpurun_out
echo "host cpus: $(nproc)"; lscpu | grep "Model name"
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_$TAG.log; [ $rc -ne 0 ] && exit $rc
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python -u bench.py --cpu-seconds 10 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log; [ $rc -ne 0 ] && exit $rc
for c in ${CONFIGS:-cfg3 cfg4}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_${c}_$TAG.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$c rc=$rc"; tail -5 gpurun_out/bench_${c}_$TAG.log; exit $rc; }
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/bench_${c}_$TAG.log') if x.startswith('{')][-1])
print('$c', d['value'], d['stage_ms'])"
done
if [ -z "$NO_TRACE" ]; then
  for c in ${TRACE_CONFIGS:-cornell}; do
    RTMI_LANES=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kt1_${c}_$TAG -o kt --output-format csv -- \
      python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/kt1_${c}_$TAG.log 2>&1
    rc=$?; echo "rocprof single-lane $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
fi
exit 0
