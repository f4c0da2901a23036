set -o pipefail
cd "$GRAFT_REPO_ROOT"
for g in 0 128 192 224 240 0; do
  RSORT_OS_GRID=$g timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/grid_$g.json 2>/dev/null || exit 11
  echo "grid=$g $(python -c "import json;d=json.loads(open('gpurun_out/grid_$g.json').read().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])")" >> gpurun_out/grid_sweep.txt
done
