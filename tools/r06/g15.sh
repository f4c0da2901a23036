# Round 6: k_ns_merge variants on config 4 (speculative slot loads; 4 / 2 workgroups per CU)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
for v in base spec mb4 specmb; do
  L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ $v != base ] && L=$E/librsort_$v.so
  RSORT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/ns_$v -o p --output-format csv -- python3 bench.py --workload config4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/ns_$v.json 2> gpurun_out/ab/ns_$v.err || exit 1
  python3 - <<PY
import csv,glob,json
d=json.loads(open('gpurun_out/ab/ns_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['device_path'])
f=glob.glob("gpurun_out/ab/ns_$v/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'ns_' in r["Name"]:
        print('  ', r["Name"][:50], r["Calls"], round(float(r["AverageNs"])/1e6,4))
PY
done
# k_onesweep without the tail barrier: config2 (keys-only passes) A/B
for r in 1 2; do for v in base ostb; do
  L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ $v != base ] && L=$E/librsort_$v.so
  RSORT_LIB=$L timeout -k 10 200 python3 bench.py --workload config2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/ostb_${v}_r$r.json 2> gpurun_out/ab/ostb_${v}_r$r.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/ab/ostb_${v}_r$r.json').read().strip().splitlines()[-1]);print('$v',$r,d['ms_per_step'],d['roofline']['avg_launch_ms'],d['kernel_ms_per_step'])"
done; done
