# Round 4 final, part E (library with the pipelined scan): tools/gpu_round.sh steps 1-7 (full GPU
# suite, smoke, default bench line, texture / config2 / config4 / check_order lines), the prefix_sum
# line and its rocprofv3 kernel stats, step 9 (PMC traffic of config3 / config2 / config4).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
bash tools/gpu_round.sh 1 7 || exit $?
timeout -k 10 300 python bench.py --workload prefix_sum > gpurun_out/bench_prefix_sum.json 2> gpurun_out/bench_prefix_sum.err || exit 33
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o ps --output-format csv -- python3 bench.py --workload prefix_sum --no-cpu-baseline > gpurun_out/prof_ps.json 2> gpurun_out/prof_ps.err || exit 34
bash tools/gpu_round.sh 9 9 || exit $?
exit 0
