# plain / range / 8-byte histogram variants: MSD tests and the two bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_msd_gpu.py tests/test_texture_gpu.py tests/test_group_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/hv_tests.log 2>&1 || exit 11
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/hv_c3.json 2> gpurun_out/hv.err || exit 12
timeout -k 10 200 python bench.py --workload config3_texture --no-cpu-baseline > gpurun_out/hv_tex.json 2>> gpurun_out/hv.err || exit 13
timeout -k 10 300 python tools/range_time.py > gpurun_out/hv_range.jsonl 2>> gpurun_out/hv.err || exit 14
