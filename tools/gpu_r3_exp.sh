# round-3: IC-resident R2 experiment (sweep library, results invalid by design); the wide-bucket
# tests; then the product library's fast GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RSORT_LIB=$PWD/exp_lib/librsort_sweep.so timeout -k 10 400 python -u tools/exp_ring.py 0 28 25 24 23 22 20 > gpurun_out/r3_exp_ring.jsonl 2> gpurun_out/r3_exp_ring.err || exit 11
timeout -k 10 600 python -u -m pytest tests/test_msd_gpu.py tests/test_large_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r3_wide.log 2>&1 || exit 12
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_gpu_fast2.log 2>&1 || exit 13
