# round-2 GPU check: new robustness / large-N tests first, then the whole -m gpu suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_robustness_gpu.py tests/test_large_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r2_new_tests.log 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r2_all_tests.log 2>&1 || exit 12
