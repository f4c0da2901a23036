# Round 6: look-back window variants (A/B in one box): first-round 6 / 8, every round 5 / 3
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in 1 2; do
  for v in base lbf6 lbf8 lb5 lb3; do
    L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ $v != base ] && L=$E/librsort_$v.so
    RSORT_LIB=$L timeout -k 10 200 python3 bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/lbf_${v}_r$r.json 2> gpurun_out/ab/lbf_${v}_r$r.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab/lbf_${v}_r$r.json').read().strip().splitlines()[-1]);print('$v',$r,d['ms_per_step'],d['roofline']['avg_launch_ms'])"
  done
done
