# Round 5: k_ns_merge A/B - HEAD (old), current without the first-fetch wait (noc), current (new).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abm2
for r in 1 2; do for v in old noc new; do
  lib=ab_lib/librsort_$v.so; [ $v = new ] && lib=webgpu-radix-sort_amd/lib/librsort.so
  RSORT_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload config4 --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/abm2/${v}_r$r.json 2> gpurun_out/abm2/${v}_r$r.err || { tail -5 gpurun_out/abm2/${v}_r$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/abm2/${v}_r$r.json').read().strip().splitlines()[-1]);print('$v',$r,d['ms_per_step'],d['value'])"
done; done
