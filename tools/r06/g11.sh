# Round 6: look-back window 4 / 8 / 16 (A/B in one box) and stamps at 16
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in 1 2; do
  for v in base lb8 lb16; do
    L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ $v != base ] && L=$E/librsort_$v.so
    RSORT_LIB=$L timeout -k 10 200 python3 bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/lbw_${v}_r$r.json 2> gpurun_out/ab/lbw_${v}_r$r.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab/lbw_${v}_r$r.json').read().strip().splitlines()[-1]);print('$v',$r,d['ms_per_step'],d['roofline']['avg_launch_ms'])"
  done
done
RSORT_LIB=$E/librsort_st16.so timeout -k 10 200 python3 tools/stamp_probe_msd.py > gpurun_out/stamps_st16.jsonl 2> gpurun_out/stamps_st16.err || { tail gpurun_out/stamps_st16.err; exit 1; }
cat gpurun_out/stamps_st16.jsonl
