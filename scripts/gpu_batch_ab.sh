cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for v in ${BATCHES:-"16:16777216:6" "24:25165824:4" "32:33554432:3"}; do
    spp=${v%%:*}; rest=${v#*:}; bs=${rest%%:*}; st=${rest#*:}
    RTMI_BATCH_SAMPLES=$bs timeout -k 10 300 python bench.py --config ${CONFIG:-cornell} --steps $st --warmup 1 --no-cpu-baseline --project-shards 0 --spp-per-step $spp > gpurun_out/batch_${spp}_$r.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/batch_${spp}_$r.log') if x.startswith('{')][-1])
print('round $r ${CONFIG:-cornell} spp/step $spp', d['value'], d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if k!='basis'})"
  done
done
