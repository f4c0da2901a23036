# full GPU suite, smoke, default bench (with CPU baseline), rocprof stats of the bench, PMC traffic
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || exit 11
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || exit 12
timeout -k 10 300 python bench.py > gpurun_out/full_bench_c3.json 2> gpurun_out/full_bench_c3.err || exit 13
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_full -o b --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/full_bench_prof.json 2> gpurun_out/full_bench_prof.err || exit 14
timeout -k 10 600 python3 tools/pmc_traffic.py config3 gpurun_out/traffic_full.json > gpurun_out/pmc_full.log 2>&1 || exit 15
