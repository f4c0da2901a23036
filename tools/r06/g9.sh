# Round 6: GPU tests of the changed paths (probe fix, tail barrier, listed tile, split grid)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_presorted_gpu.py tests/test_msd_gpu.py tests/test_region_gpu.py tests/test_split_gpu.py tests/test_sort_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t9.log 2>&1 || { tail -40 gpurun_out/t9.log; exit 1; }
tail -3 gpurun_out/t9.log
for w in config3 config4 config2; do
  timeout -k 10 200 python3 bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b9_$w.json 2> gpurun_out/b9_$w.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/b9_$w.json').read().strip().splitlines()[-1]);print('$w',d['ms_per_step'],d['value'],d['roofline'])"
done
