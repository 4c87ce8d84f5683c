#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
# Round check (smoke, -m gpu, bench lines for every config) plus rocprofv3 kernel traces of CFG3 and CFG4.
TAG=r01i CONFIGS="cfg3 cfg4 cfg5" bash scripts/gpu_round.sh || exit 1
for c in cfg3 cfg4; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${c}_r01i -o kt --output-format csv -- \
    python3 bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/kt_${c}_r01i.log 2>&1
  rc=$?; echo "kt $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
