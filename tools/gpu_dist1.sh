# multi-GPU paths at world size 1: tests + distributed bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_distributed.py tests/test_group_gpu.py tests/test_records_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/dist1_tests.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --distributed --no-cpu-baseline > gpurun_out/r2_bench_dist1.json 2> gpurun_out/r2_bench_dist1.err || exit 12
