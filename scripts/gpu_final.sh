#!/bin/bash
# Round evidence of one build, in GPU calls of their own (PART=a / b / c); stops at the first failure.
#   a: smoke, the -m gpu suite, single-lane kernel traces + PMC counters of Cornell / CFG3 / CFG4 / CFG5
#   b: >= 8-step bench lines of every BASELINE config (the default line with the CPU baseline; CFG4 / CFG5 lines with
#      the 8-shard tile-efficiency projection)
#   c: where the Cornell kernels wait (SQ wait / LDS / SMEM counters, gpu_pmc_wait.sh)
#   rp: the default bench command under rocprofv3 --kernel-trace --stats
#   ab: a, then b with a's counters installed
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-r05a}
case "${PART:-a}" in
a)
  timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke_$TAG.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 2 gpurun_out/pytest_gpu_$TAG.log; [ $rc -ne 0 ] && exit $rc
  TAG=$TAG CONFIGS="${CONFIGS:-cornell cfg3 cfg4 cfg5}" bash scripts/gpu_counters.sh || exit 1
  ;;
b)
  timeout -k 10 600 python -u bench.py --steps 8 --warmup 2 --cpu-seconds 12 > gpurun_out/bench_default_$TAG.log 2>&1
  rc=$?; echo "default bench rc=$rc"; tail -n 1 gpurun_out/bench_default_$TAG.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
  TAG=$TAG STEPS=8 CONFIGS="${CONFIGS:-cornell cfg3 cfg4 cfg5}" bash scripts/gpu_bench_cfgs.sh || exit 1
  ;;
c)
  CFG=cornell TAG=$TAG bash scripts/gpu_pmc_wait.sh || exit 1
  ;;
rp)  # the default bench command itself under rocprofv3 --kernel-trace --stats (its summary goes to profiles/)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rp_default_$TAG -o rp --output-format csv -- \
    python3 bench.py --steps 8 --warmup 2 --cpu-seconds 5 > gpurun_out/bench_default_under_rocprof_$TAG.log 2>&1
  rc=$?; echo "rocprof default rc=$rc"; tail -n 1 gpurun_out/bench_default_under_rocprof_$TAG.log | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
  ;;
ab)  # a, the new counters installed into this copy's profiles/ (the bench reads them), then b
  PART=a TAG=$TAG bash scripts/gpu_final.sh || exit 1
  for c in ${CONFIGS:-cornell cfg3 cfg4 cfg5}; do cp gpurun_out/cnt_${c}_$TAG.counters.json profiles/counters_$c.json || exit 1; done
  PART=b TAG=$TAG bash scripts/gpu_final.sh || exit 1
  ;;
esac
exit 0
