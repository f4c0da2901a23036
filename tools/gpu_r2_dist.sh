# records API + multi-GPU path at world 1 + default bench + distributed bench (world 1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_records_gpu.py tests/test_distributed.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2_records_tests.log 2>&1 || exit 11
timeout -k 10 300 python bench.py > gpurun_out/r2_bench_c3.json 2> gpurun_out/r2_bench_c3.err || exit 12
timeout -k 10 300 python bench.py --distributed > gpurun_out/r2_bench_dist1.json 2> gpurun_out/r2_bench_dist1.err || exit 13
