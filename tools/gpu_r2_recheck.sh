# re-entry check of a fresh build: full GPU suite, smoke, default bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rc_gpu_tests.log 2>&1 || exit 11
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc_smoke.log 2>&1 || exit 12
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/rc_bench_c3.json 2> gpurun_out/rc_bench.err || exit 13
timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline > gpurun_out/rc_bench_c2.json 2>> gpurun_out/rc_bench.err || exit 14
