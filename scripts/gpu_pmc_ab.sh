#!/bin/bash
# SQ instruction mix per kernel for each A/B variant (computational_ray_tracer_amd/lib/variants/*.so), one lane,
# one PMC pass per variant (counter groups never combined with tracing).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
GRP=${GRP:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"}
for so in computational_ray_tracer_amd/lib/variants/*.so; do
  n=$(basename $so .so)
  RTMI_LANES=1 RTMI_LIB=$PWD/$so timeout -k 10 300 rocprofv3 --pmc $GRP -d gpurun_out/pmcab_$n -o pmc \
    --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} \
    > gpurun_out/pmcab_$n.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$n rc=$rc"; exit $rc; }
  echo "== $n"
  python3 tools/pmc_summary.py $(find gpurun_out/pmcab_$n -name "*counter_collection.csv") | grep -E "k_trace|k_path_shade"
done
