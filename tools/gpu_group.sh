# multi-GPU C ABI (rs_group_*): Python and Node GPU tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_node.py tests/test_group_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2_group_tests.log 2>&1 || exit 11
