# Round 6: MSD pass 0 over 32K-record tiles (k_onesweep SR = 2) vs 16K (k_msd_pass), per-kernel times
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
for v in base sr2; do
  L=$PWD/webgpu-radix-sort_amd/lib/librsort.so; [ $v != base ] && L=$E/librsort_$v.so
  RSORT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/sr2_$v -o p --output-format csv -- python3 bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/sr2_$v.json 2> gpurun_out/ab/sr2_$v.err || exit 1
  python3 - <<PY
import csv,glob,json
d=json.loads(open('gpurun_out/ab/sr2_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])
f=glob.glob("gpurun_out/ab/sr2_$v/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'onesweep' in r["Name"] or 'msd_pass' in r["Name"]:
        print('  ', r["Name"][:70], r["Calls"], round(float(r["AverageNs"])/1e6,4))
PY
done
