# round-2 measurements: host-ASan driver, run-length probe, rocprof kernel stats of the bench,
# PMC traffic (config3, config2), bench lines for config2 / config4 / texture
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 timeout -k 10 300 ./tools/asan_driver > gpurun_out/asan_driver.log 2>&1 || exit 11
timeout -k 10 200 ./tools/line_probe runs > gpurun_out/line_probe_runs.jsonl 2> gpurun_out/line_probe_runs.err || exit 12
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o b --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r02_bench_prof.json 2> gpurun_out/r02_bench_prof.err || exit 13
timeout -k 10 600 python3 tools/pmc_traffic.py config3 gpurun_out/traffic_c3.json > gpurun_out/pmc.log 2>&1 || exit 14
timeout -k 10 600 python3 tools/pmc_traffic.py config2 gpurun_out/traffic_c2.json >> gpurun_out/pmc.log 2>&1 || exit 15
timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > gpurun_out/r02_bench_c2.json 2> gpurun_out/r02_bench_c2.err || exit 16
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline > gpurun_out/r02_bench_c4.json 2> gpurun_out/r02_bench_c4.err || exit 17
timeout -k 10 300 python bench.py --workload config3_texture --no-cpu-baseline > gpurun_out/r02_bench_tex.json 2> gpurun_out/r02_bench_tex.err || exit 18
