# Round 6: k_hist16_in with the group's adds batched (FLY 6 / 3) vs the product
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
for v in base hb2 hb3 hb4 f3; do
  L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ $v != base ] && L=$E/librsort_$v.so
  RSORT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/h16_$v -o p --output-format csv -- python3 bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/h16_$v.json 2> gpurun_out/ab/h16_$v.err || exit 1
  python3 - <<PY
import csv,glob,json
d=json.loads(open('gpurun_out/ab/h16_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['device_path'])
f=glob.glob("gpurun_out/ab/h16_$v/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'hist16' in r["Name"]:
        print('  ', r["Name"][:70], r["Calls"], round(float(r["AverageNs"])/1e6,4))
PY
done
