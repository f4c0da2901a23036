# Round 6: per-kernel split of the XCD-local claims (rocprof kernel stats per variant)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/prof
for v in 0 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/xcd$v -o b --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --plan-debug xcd=$v > gpurun_out/prof/xcd$v.json 2> gpurun_out/prof/xcd$v.err || exit 1
done
python3 - <<'PY'
import csv,glob
for v in range(4):
    f=glob.glob(f"gpurun_out/prof/xcd{v}/**/*kernel_stats.csv",recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "msd_pass" in r["Name"] or "bucket_sort" in r["Name"] or "hist16_in" in r["Name"]:
            print(v, r["Name"][:90], r["Calls"], round(float(r["AverageNs"])/1e6,4))
PY
