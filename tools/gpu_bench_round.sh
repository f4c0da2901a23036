set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 11
timeout -k 10 300 python bench.py --workload config3_texture --no-cpu-baseline > gpurun_out/bench_tex.json 2> gpurun_out/bench_tex.err || exit 12
timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 13
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 14
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o b --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit 15
timeout -k 10 600 python3 tools/pmc_traffic.py config3 gpurun_out/traffic_c3.json > gpurun_out/pmc.log 2>&1 || exit 16
timeout -k 10 600 python3 tools/pmc_traffic.py config2 gpurun_out/traffic_c2.json >> gpurun_out/pmc.log 2>&1 || exit 17
