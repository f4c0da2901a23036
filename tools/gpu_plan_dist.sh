# the MSD plan spread over the histogram reduction: every MSD test, texture / records / group tests,
# bench lines for config3 / config2 / texture
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_msd_gpu.py tests/test_records_gpu.py tests/test_group_gpu.py tests/test_texture_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pd_tests.log 2>&1 || exit 11
: > gpurun_out/pd.jsonl
for wl in config3 config2 config3_texture config2 config3; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 20 >> gpurun_out/pd.jsonl 2>> gpurun_out/pd.err || exit 12
done
