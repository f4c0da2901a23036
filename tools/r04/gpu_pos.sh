# Round 4: the bucket pass through 4-byte (key bits, position) staging at 4 / 5 / 6 workgroups per
# CU against the 8-byte record staging (3 per CU), config3 A/B (bench verifies the last batch).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in 1 2; do
  for v in base pos4 pos5 pos6; do
    if [ $v = base ]; then L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; else L=$E/librsort_$v.so; fi
    RSORT_LIB=$L timeout -k 10 200 python bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/c3_${v}_r$r.json 2> gpurun_out/c3_${v}_r$r.err || exit 11
  done
done
RSORT_LIB=$E/librsort_pos5.so timeout -k 10 200 python bench.py --workload config3_texture --no-cpu-baseline --steps 10 > gpurun_out/tex_pos5.json 2> gpurun_out/tex_pos5.err || exit 12
exit 0
