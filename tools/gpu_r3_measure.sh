# round-3 measurements: a rank's local work at config-5 shape, the bench lines (config3 default,
# config2, config4, --distributed world 1), and the rocprofv3 kernel stats of the default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u tools/rank_model.py > gpurun_out/r3_rank_model.json 2> gpurun_out/r3_rank_model.err || exit 11
timeout -k 10 300 python -u bench.py > gpurun_out/r3_bench_c3.json 2> gpurun_out/r3_bench_c3.err || exit 12
timeout -k 10 300 python -u bench.py --workload config2 --no-cpu-baseline > gpurun_out/r3_bench_c2.json 2> gpurun_out/r3_bench_c2.err || exit 13
timeout -k 10 300 python -u bench.py --workload config4 --no-cpu-baseline > gpurun_out/r3_bench_c4.json 2> gpurun_out/r3_bench_c4.err || exit 14
timeout -k 10 300 python -u bench.py --distributed --no-cpu-baseline > gpurun_out/r3_bench_dist1.json 2> gpurun_out/r3_bench_dist1.err || exit 15
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r3c3 -- python3 bench.py --no-cpu-baseline > gpurun_out/r3_bench_c3_under_rocprof.json 2> gpurun_out/r3_prof.err || exit 16
