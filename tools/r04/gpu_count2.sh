# Round 4: split count in half tiles (two workgroups per CU): split suite, config4 line + trace.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_split.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline --steps 10 > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 --output-format csv -- python3 bench.py --workload config4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prof_c4.log 2>&1 || exit 16
exit 0
