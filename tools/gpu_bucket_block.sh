# bucket-kernel workgroup size sweep (RSORT_BUCKET_BLOCK), alternated, config3 bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/bb.jsonl
for rep in 1 2; do
  for bb in 256 128; do
    echo "{\"bb\": $bb}" >> gpurun_out/bb.jsonl
    RSORT_BUCKET_BLOCK=$bb timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 >> gpurun_out/bb.jsonl 2>> gpurun_out/bb.err || exit 11
  done
done
RSORT_BUCKET_BLOCK=128 timeout -k 10 300 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bb_tests128.log 2>&1 || exit 12
