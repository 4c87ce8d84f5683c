#!/bin/bash
# PMC passes (SQ instruction / wait mix, L2 hit rate) for one bench config: CFG=cfg3 bash scripts/gpu_pmc_cfg.sh
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CFG=${CFG:-cfg3}
mkdir -p gpurun_out
B="python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --spp-per-step ${SPP:-2}"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp -d gpurun_out/pmc_${CFG}_$i -o pmc --output-format csv -- $B > gpurun_out/pmc_${CFG}_$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc_${CFG}_*/pmc_counter_collection.csv
