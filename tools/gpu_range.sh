# key-range hybrid MSD path (records -> arrays; group regions): tests, then a group-sort timing
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_msd_gpu.py tests/test_group_gpu.py tests/test_records_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/range_tests.log 2>&1 || exit 11
