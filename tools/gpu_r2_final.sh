# round-2 closing measurements: full GPU suite, smoke, ASan driver, default bench (with CPU
# baseline), the other workloads, rocprof stats of the bench, PMC traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
true
true
ASAN_OPTIONS=halt_on_error=1 LSAN_OPTIONS=suppressions=tools/lsan.supp:print_suppressions=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 timeout -k 10 300 ./tools/asan_driver > gpurun_out/fin_asan.log 2>&1 || exit 13
timeout -k 10 300 python bench.py > gpurun_out/fin_bench_c3.json 2> gpurun_out/fin_bench.err || exit 14
timeout -k 10 200 python bench.py --workload config3_texture --no-cpu-baseline > gpurun_out/fin_bench_tex.json 2>> gpurun_out/fin_bench.err || exit 15
timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline > gpurun_out/fin_bench_c2.json 2>> gpurun_out/fin_bench.err || exit 16
timeout -k 10 200 python bench.py --workload config4 --no-cpu-baseline > gpurun_out/fin_bench_c4.json 2>> gpurun_out/fin_bench.err || exit 17
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fin -o b --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/fin_bench_prof.json 2> gpurun_out/fin_bench_prof.err || exit 18
timeout -k 10 600 python3 tools/pmc_traffic.py config3 gpurun_out/traffic_fin.json > gpurun_out/fin_pmc.log 2>&1 || exit 19
