# Round 5: config3 / texture with branch-free loads in every bucket tile (buf) against the library (new).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/abbuf
for r in 1 2; do for w in config3 config3_texture; do for v in new buf; do
  lib=ab_lib/librsort_$v.so; [ $v = new ] && lib=webgpu-radix-sort_amd/lib/librsort.so
  RSORT_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/abbuf/${w}_${v}_r$r.json 2> gpurun_out/abbuf/${w}_${v}_r$r.err || { tail -5 gpurun_out/abbuf/${w}_${v}_r$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/abbuf/${w}_${v}_r$r.json').read().strip().splitlines()[-1]);print('$w','$v',$r,d['ms_per_step'],d['extra'].get('bucket_pass',{}).get('ms_per_sort'))"
done; done; done
