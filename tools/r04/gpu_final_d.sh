# Round 4 final, part D (library with the reordered scan look-back): the prefix_sum line and its
# rocprofv3 kernel stats, then tools/gpu_round.sh steps 8-12 (rocprof of the default line, PMC
# traffic, rank model, 2-rank rehearsal, ASan driver).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload prefix_sum > gpurun_out/bench_prefix_sum.json 2> gpurun_out/bench_prefix_sum.err || exit 33
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o ps --output-format csv -- python3 bench.py --workload prefix_sum --no-cpu-baseline > gpurun_out/prof_ps.json 2> gpurun_out/prof_ps.err || exit 34
bash tools/gpu_round.sh 8 12 || exit $?
exit 0
