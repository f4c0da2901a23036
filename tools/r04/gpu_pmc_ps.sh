# Round 4: PMC HBM traffic of the single-pass scan (k_scan_lookback, 2^28 u32), then the prefix_sum
# bench line reading it back.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python3 tools/pmc_traffic.py prefix_sum gpurun_out/traffic_prefix_sum.json > gpurun_out/pmc_prefix_sum.log 2>&1 || exit 11
timeout -k 10 300 python bench.py --workload prefix_sum --traffic-json gpurun_out/traffic_prefix_sum.json > gpurun_out/bench_prefix_sum.json 2> gpurun_out/bench_prefix_sum.err || exit 12
exit 0
