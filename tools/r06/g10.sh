# Round 6: late look-back-wave loads (A/B in one box) and phase stamps of both
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in 1 2 3; do
  for v in base lbl; do
    L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ $v = lbl ] && L=$E/librsort_lbl.so
    RSORT_LIB=$L timeout -k 10 200 python3 bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/lbl_${v}_r$r.json 2> gpurun_out/ab/lbl_${v}_r$r.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab/lbl_${v}_r$r.json').read().strip().splitlines()[-1]);print('$v',$r,d['ms_per_step'],d['roofline']['avg_launch_ms'])"
  done
done
for v in st stl; do
  RSORT_LIB=$E/librsort_$v.so timeout -k 10 200 python3 tools/stamp_probe_msd.py > gpurun_out/stamps_$v.jsonl 2> gpurun_out/stamps_$v.err || { tail gpurun_out/stamps_$v.err; exit 1; }
  echo $v; cat gpurun_out/stamps_$v.jsonl
done
