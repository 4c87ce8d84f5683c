cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pt.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2 3; do for so in computational_ray_tracer_amd/lib/variants/*.so; do n=$(basename $so .so)
  RTMI_LIB=$PWD/$so timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$n.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/ab_$n.log') if x.startswith('{')][-1])
print('round $round', '$n', d['value'], d['roofline']['avg_launch_ms'])"
done; done
