#!/bin/bash
# PMC pass(es) for the path-mode kernels: SQ instruction/stall mix (one pass per counter group).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/${TAG}_$i -o pmc --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --spp-per-step 4 > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?; echo "pmc group $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
