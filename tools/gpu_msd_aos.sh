# hybrid MSD path for the texture (records) layout: its tests, the texture suite, a bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_msd_gpu.py tests/test_texture_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/aos_tests.log 2>&1 || exit 11
timeout -k 10 200 python bench.py --workload config3_texture > gpurun_out/aos_bench.json 2> gpurun_out/aos_bench.err || exit 12
RSORT_MSD=0 timeout -k 10 200 python bench.py --workload config3_texture > gpurun_out/aos_bench_lsd.json 2>> gpurun_out/aos_bench.err || exit 13
