# Round 5 A/B: k_ns_merge workgroup size (512 / 256 / 1024 threads per tile), config4, two reps each.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab_nt
for r in 1 2; do for v in m512 m256 m1024; do
  RSORT_LIB=$PWD/ab_lib/librsort_$v.so timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline \
    > gpurun_out/ab_nt/${v}_r$r.json 2> gpurun_out/ab_nt/${v}_r$r.err || exit 1
done; done
exit 0
