# Round 4 final, part A: split count (half tiles) checks, then tools/gpu_round.sh steps 1-7 (full GPU
# suite, smoke, default bench line, texture / config2 / config4 / check_order lines).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_split_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_split.log 2>&1 || exit 31
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o c4 --output-format csv -- python3 bench.py --workload config4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/prof_c4.log 2>&1 || exit 32
bash tools/gpu_round.sh 1 7
