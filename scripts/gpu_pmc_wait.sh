#!/bin/bash
# Where the Cornell (configs[1]) kernels wait: single-lane PMC passes of one bench step, each pass its own run.
#   CFG=cornell TAG=r05a bash scripts/gpu_pmc_wait.sh  -> gpurun_out/pmcw_<cfg>_<tag>.txt
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
CFG=${CFG:-cornell}; TAG=${TAG:-r04}
B="python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --project-shards 0"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_FLAT TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  RTMI_LANES=1 timeout -s KILL 240 rocprofv3 --pmc $grp -d gpurun_out/pmcw_${CFG}_${TAG}_$i -o pmc --output-format csv -- $B > gpurun_out/pmcw_${CFG}_${TAG}_$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmcw_${CFG}_${TAG}_$i.log; exit $rc; }
done
python3 tools/pmc_summary.py gpurun_out/pmcw_${CFG}_${TAG}_*/pmc*/*counter_collection.csv gpurun_out/pmcw_${CFG}_${TAG}_*/*counter_collection.csv 2>/dev/null > gpurun_out/pmcw_${CFG}_${TAG}.txt
cat gpurun_out/pmcw_${CFG}_${TAG}.txt | cut -c1-600
