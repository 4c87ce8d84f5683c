#!/bin/bash
# GPU-box profiling of the bench workload: rocprofv3 kernel-trace stats, separate PMC passes (FETCH_SIZE,
# WRITE_SIZE, two SQ instruction-mix groups — never combined with other tracing), then the bench line itself.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o kt --output-format csv -- \
  $B > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof kt rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$TAG -o pmc --output-format csv -- \
  $B > gpurun_out/pmc_fetch_$TAG.log 2>&1
rc=$?; echo "rocprof fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$TAG -o pmc --output-format csv -- \
  $B > gpurun_out/pmc_write_$TAG.log 2>&1
rc=$?; echo "rocprof write rc=$rc"; [ $rc -ne 0 ] && exit $rc
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp -d gpurun_out/pmc_sq${i}_$TAG -o pmc --output-format csv -- \
    $B > gpurun_out/pmc_sq${i}_$TAG.log 2>&1
  rc=$?; echo "pmc sq group $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log; exit $rc
