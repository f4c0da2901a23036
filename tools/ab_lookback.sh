# A/B of the one-sweep look-back window (RS_LOOKBACK 2/4/8/16): config3 and config2 bench lines per
# variant library (built by hand into webgpu-radix-sort_amd/lib/lbvar/), alternated twice
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for v in lb4 lb8 lb16 lb2; do
    for w in config3 config2; do
      RSORT_LIB=$PWD/webgpu-radix-sort_amd/lib/lbvar/librsort_$v.so timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --steps 20 > gpurun_out/lb_${v}_${w}_r$r.json 2>/dev/null || exit 1
    done
  done
done
