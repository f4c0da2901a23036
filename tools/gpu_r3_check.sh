# round-3 GPU check: the large-N tests (new default-route max-count case), the whole -m gpu suite,
# then one default bench line.  Each GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_large_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_large.log 2>&1 || exit 11
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_gpu_fast.log 2>&1 || exit 12
timeout -k 10 300 python -u bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || exit 13
