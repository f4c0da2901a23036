# Round 6: 32-bit look-back status words in k_msd_pass (memset before each pass), windows 4 / 6 / 8
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/ab
E=$PWD/webgpu-radix-sort_amd/lib/exp
RSORT_LIB=$E/librsort_st32.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_msd_gpu.py tests/test_region_gpu.py > gpurun_out/ab/st32_tests.log 2>&1 || { tail -30 gpurun_out/ab/st32_tests.log; exit 1; }
tail -2 gpurun_out/ab/st32_tests.log
for r in 1 2; do for v in base st32 st32w6 st32w8; do
  L=$E/librsort_$v.so
  RSORT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/st_${v}_r$r -o p --output-format csv -- python3 bench.py --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab/st_${v}_r$r.json 2> gpurun_out/ab/st_${v}_r$r.err || exit 1
  python3 - <<PY
import csv,glob,json
d=json.loads(open('gpurun_out/ab/st_${v}_r$r.json').read().strip().splitlines()[-1]); print('$v', $r, d['ms_per_step'], d['kernel_ms_per_step'])
f=glob.glob("gpurun_out/ab/st_${v}_r$r/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'msd_pass' in r["Name"] or 'fillBuffer' in r["Name"]:
        print('  ', r["Name"][:50], r["Calls"], round(float(r["AverageNs"])/1e6,4))
PY
done; done
