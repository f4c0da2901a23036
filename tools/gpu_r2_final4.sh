# round-2 closing check on the final build: full GPU suite, smoke, default bench (CPU baseline),
# the other workloads, rocprof kernel stats of config3 and config2
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f4_gpu_tests.log 2>&1 || exit 11
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f4_smoke.log 2>&1 || exit 12
timeout -k 10 300 python bench.py > gpurun_out/f4_bench_c3.json 2> gpurun_out/f4_bench.err || exit 13
timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/f4_bench_c2.json 2>> gpurun_out/f4_bench.err || exit 14
timeout -k 10 200 python bench.py --workload config3_texture --no-cpu-baseline > gpurun_out/f4_bench_tex.json 2>> gpurun_out/f4_bench.err || exit 15
timeout -k 10 200 python bench.py --workload config4 --no-cpu-baseline > gpurun_out/f4_bench_c4.json 2>> gpurun_out/f4_bench.err || exit 16
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f4_c3 -o b --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/f4_bench_c3_prof.json 2>> gpurun_out/f4_bench.err || exit 17
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f4_c2 -o b --output-format csv -- python3 bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/f4_bench_c2_prof.json 2>> gpurun_out/f4_bench.err || exit 18
