# Round 6: traffic attribution of the pass kernels (config2 keys-only k_onesweep, config3 k_msd_pass):
# base / no look-back status reads / sequential writes (no run seams) / both; PMC bytes + durations
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/attr
E=$PWD/webgpu-radix-sort_amd/lib/exp
export RS_PROF_NOCHECK=1
for wl in config2 config3; do for v in base nolb seq nolbseq; do
  RSORT_LIB=$E/librsort_$v.so timeout -k 10 300 python3 tools/pmc_traffic.py $wl gpurun_out/attr/traffic_$v.json > gpurun_out/attr/${wl}_$v.log 2>&1 || { tail -5 gpurun_out/attr/${wl}_$v.log; exit 1; }
  RSORT_LIB=$E/librsort_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/attr/k_${wl}_$v -o p --output-format csv -- python3 tools/prof_driver.py $wl 4 > /dev/null 2>&1 || exit 1
  python3 - <<PY
import csv,glob,json
d=json.load(open('gpurun_out/attr/traffic_$v.json'))['$wl']
f=glob.glob("gpurun_out/attr/k_${wl}_$v/**/*kernel_stats.csv",recursive=True)[0]
ms={r["Name"][:40]:round(float(r["AverageNs"])/1e6,4) for r in csv.DictReader(open(f)) if ('msd_pass' in r["Name"] or 'k_onesweep' in r["Name"]) and float(r["AverageNs"])>20000}
print('$wl','$v','rd',round(d['scatter_read_bytes_per_launch']/1e6,1),'wr',round(d['scatter_write_bytes_per_launch']/1e6,1),'alg',d['scatter_algorithmic_bytes_per_launch']/1e6,'x',d['scatter_traffic_over_algorithmic'],ms)
PY
done; done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_region_gpu.py tests/test_split_gpu.py tests/test_group_gpu.py tests/test_distributed.py > gpurun_out/attr/region_tests.log 2>&1 || { tail -30 gpurun_out/attr/region_tests.log; exit 1; }
tail -1 gpurun_out/attr/region_tests.log
timeout -k 10 300 python3 tools/rank_model.py --reps 10 > gpurun_out/attr/rank_model.json 2>gpurun_out/attr/rank_model.err || exit 1
cat gpurun_out/attr/rank_model.json
