# Round 4: striped single-pass scan - parity suites and the prefix_sum bench line (+ trace).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_robustness_gpu.py tests/test_property_gpu.py tests/test_sort_gpu.py -k "scan or prefix" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_scan.log 2>&1 || exit 12
timeout -k 10 300 python bench.py --workload prefix_sum --no-cpu-baseline --steps 20 > gpurun_out/ps.json 2> gpurun_out/ps.err || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ps -o ps --output-format csv -- python3 bench.py --workload prefix_sum --no-cpu-baseline --steps 10 > gpurun_out/prof_ps.log 2>&1 || exit 15
exit 0
