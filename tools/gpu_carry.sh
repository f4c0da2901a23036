# line-carry k_onesweep: KV parity tests, then the config3 bench with the carry off / on
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sort_gpu.py tests/test_records_gpu.py tests/test_texture_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -k "config3 or config4 or onesweep or duplicate or records or texture or sizes or rank_modes" > gpurun_out/carry_tests.log 2>&1 || exit 11
RSORT_CARRY=0 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/carry_bench_off.json 2> gpurun_out/carry_bench_off.err || exit 12
RSORT_CARRY=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/carry_bench_on.json 2> gpurun_out/carry_bench_on.err || exit 13
