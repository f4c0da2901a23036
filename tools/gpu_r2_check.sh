# round-2 full check: whole -m gpu suite, smoke, default bench, config2 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_all_tests.log 2>&1 || exit 11
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 || exit 12
timeout -k 10 300 python bench.py > gpurun_out/r2_bench_c3.json 2> gpurun_out/r2_bench_c3.err || exit 13
timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > gpurun_out/r2_bench_c2.json 2> gpurun_out/r2_bench_c2.err || exit 14
