cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
export RTMI_RGBSPEC_TABLE=$PWD/computational_ray_tracer_amd/data/srgb64.rgbspec
for r in 0 16 4; do
  for c in cfg3 cfg4; do
    RTMI_LIB=$PWD/computational_ray_tracer_amd/lib/variants/simd.so RTMI_REFILL=$r RTMI_LANES=1 timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --project-shards 0 > gpurun_out/simd_${c}_$r.log 2>&1 || exit 1
    echo "$c refill=$r"; grep SIMD gpurun_out/simd_${c}_$r.log | tail -1
  done
done
