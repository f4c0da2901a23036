set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 11
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 12
timeout -k 10 400 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 13
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 14
