# round-3: the bucket-tile choice for large populations (256 x 34 / 1024 x 17 8-byte staging,
# wide 1024 x 34) through the rank model; then the hybrid-path tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/rank_model.py --reps 5 > gpurun_out/r3_tiles.json 2> gpurun_out/r3_tiles.err || exit 11
timeout -k 10 600 python -u -m pytest tests/test_msd_gpu.py tests/test_large_gpu.py tests/test_group_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r3_tiles_tests.log 2>&1 || exit 12
