set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_sort_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "check_order or onesweep or config4" > gpurun_out/gpu_iter_tests.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --workload config4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 12
timeout -k 10 600 python tools/sweep.py base base@RSORT_ONESWEEP=1 > gpurun_out/sweep_iter.jsonl 2>&1 || exit 13
