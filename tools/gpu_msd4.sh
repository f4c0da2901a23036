# plan-first hybrid MSD path: its tests, bench lines for both layouts, rocprof kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_msd_gpu.py tests/test_texture_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/m4_tests.log 2>&1 || exit 11
timeout -k 10 200 python bench.py > gpurun_out/m4_bench.json 2> gpurun_out/m4_bench.err || exit 12
timeout -k 10 200 python bench.py --workload config3_texture > gpurun_out/m4_bench_tex.json 2>> gpurun_out/m4_bench.err || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_m4 -o m --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/m4_bench_prof.json 2>> gpurun_out/m4_bench.err || exit 14
