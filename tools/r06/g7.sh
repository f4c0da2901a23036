# Round 6: no-trailing-barrier A/B, k_msd_pass phase stamps, then the presorted fault diagnosis
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in 1 2; do
  for v in base ntb; do
    L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ $v = ntb ] && L=$E/librsort_ntb.so
    RSORT_LIB=$L timeout -k 10 200 python3 bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/ntb_${v}_r$r.json 2> gpurun_out/ab/ntb_${v}_r$r.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/ab/ntb_${v}_r$r.json').read().strip().splitlines()[-1]);print('$v',$r,d['ms_per_step'],d['roofline']['avg_launch_ms'])"
  done
done
RSORT_LIB=$E/librsort_st.so timeout -k 10 200 python3 tools/stamp_probe_msd.py > gpurun_out/stamps_msd.jsonl 2> gpurun_out/stamps_msd.err || { tail gpurun_out/stamps_msd.err; exit 1; }
cat gpurun_out/stamps_msd.jsonl
bash tools/r06/g6.sh
