# A/B of k_hist16_in's loads in flight per thread (RS_H16_FLY 3/5/15): config3 and config2 bench
# lines per variant library (built by hand into webgpu-radix-sort_amd/lib/h16var/), alternated twice
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for v in f5 f15 f3; do
    for w in config3 config2; do
      RSORT_LIB=$PWD/webgpu-radix-sort_amd/lib/h16var/librsort_$v.so timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 20 > gpurun_out/h16_${v}_${w}_r$r.json 2>/dev/null || exit 1
    done
  done
done
