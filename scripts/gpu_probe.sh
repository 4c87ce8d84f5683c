#!/bin/bash
# Probe: the counter names this box offers, instruction-cache and L2 counters of the hot kernels (single lane,
# one bench step per config, every pass its own run), and a default bench line for the box.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-probe}
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/avail_$TAG.txt 2>&1
echo "list-avail rc=$?"
has() { grep -qw "$1" gpurun_out/avail_$TAG.txt; }
pick() { local o=""; for c in "$@"; do has "${c%_sum}" && o="$o $c"; done; echo $o; }
G1=$(pick SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE)
G2=$(pick SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY)
G3=$(pick TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum)
echo "groups: [$G1] [$G2] [$G3]"
for CFG in ${CONFIGS:-cornell cfg3}; do
  B="python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline --project-shards 0"
  i=0
  for grp in "$G1" "$G2" "$G3"; do
    i=$((i+1)); [ -z "$grp" ] && continue
    RTMI_LANES=1 timeout -s KILL 240 rocprofv3 --pmc $grp -d gpurun_out/pmc_${CFG}_${TAG}_$i -o pmc --output-format csv -- $B \
      > gpurun_out/pmc_${CFG}_${TAG}_$i.log 2>&1
    rc=$?; echo "$CFG pmc group $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc_${CFG}_${TAG}_$i.log; exit $rc; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${CFG}_${TAG}_*/*counter_collection.csv > gpurun_out/pmc_${CFG}_${TAG}.txt
done
timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
echo "bench rc=$?"; tail -n 1 gpurun_out/bench_$TAG.log | cut -c1-200
exit 0
