# round-3: the 52 B/key multi-GPU flow (16-bit tables, per-byte chunks, region sorts) on virtual
# ranks; BASELINE config 5's full shape (8 x 2^28 KV); then the fast GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_group_gpu.py tests/test_distributed.py tests/test_node.py -m "gpu and not slow" -x -v --timeout 240 --timeout-method thread > gpurun_out/r3_group.log 2>&1 || exit 11
timeout -k 10 500 python -u -m pytest tests/test_group_gpu.py -m "gpu and slow" -x -v --timeout 400 --timeout-method thread > gpurun_out/r3_config5.log 2>&1 || exit 12
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 240 --timeout-method thread > gpurun_out/r3_gpu_fast3.log 2>&1 || exit 13
