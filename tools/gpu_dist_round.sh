set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_distributed.py tests/test_sort_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rccl or histogram or partition" > gpurun_out/gpu_dist_tests.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --distributed --steps 10 --warmup 3 > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err || exit 12
