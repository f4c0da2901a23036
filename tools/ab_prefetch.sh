# A/B of k_onesweep's next-tile load placement (RS_PREFETCH 0/1/2) and the early ticket
# (RS_EARLY_TICKET=1) on the hybrid path: config3 bench lines per variant library (built by hand
# into webgpu-radix-sort_amd/lib/pfvar/), alternated twice
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for v in p0 p1 p2 et; do
    RSORT_LIB=$PWD/webgpu-radix-sort_amd/lib/pfvar/librsort_$v.so timeout -k 10 200 python bench.py --workload config3 --no-cpu-baseline --steps 20 > gpurun_out/pf_${v}_r$r.json 2>/dev/null || exit 1
  done
done
