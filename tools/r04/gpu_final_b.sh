# Round 4 final, part B: tools/gpu_round.sh steps 8-12 (rocprof of the default line, PMC traffic,
# rank model, 2-rank rehearsal, ASan driver) + the prefix_sum line.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload prefix_sum > gpurun_out/bench_prefix_sum.json 2> gpurun_out/bench_prefix_sum.err || exit 33
bash tools/gpu_round.sh 8 12 || exit $?
exit 0
