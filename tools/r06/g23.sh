# Round 6: config2 (keys-only k_onesweep, 512 x 32 tiles, two workgroups per CU) look-back windows 4/6/8/12
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
for r in 1 2 3; do for v in base w6 w8 w12; do
  RSORT_LIB=$E/librsort_$v.so timeout -k 10 300 python3 bench.py --workload config2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/lw_${v}_r$r.json 2>gpurun_out/ab/lw_${v}_r$r.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ab/lw_${v}_r$r.json').read().strip().splitlines()[-1]);print('bench $v',$r,d['ms_per_step'],d['roofline']['avg_launch_ms'],d['kernel_ms_per_step'])"
done; done
