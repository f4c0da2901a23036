# bucket-kernel sweep: minimum waves per SIMD (RSORT_BUCKET_MW) and tile size (RSORT_BUCKET_SIGMA /
# RSORT_BUCKET_PAD pick KPT 18 or 17 at 2^28), persistent grid multiple (RSORT_BUCKET_WAVES;
# 1000 = one workgroup per bucket); config3 bench lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/bb.jsonl
for rep in 1 2; do
  for cfg in 1:6:64:1000 3:6:64:1000 3:4:0:1000 4:4:0:1000 3:6:64:1 4:4:0:1; do
    IFS=: read mw sig pad wv <<< "$cfg"
    echo "{\"cfg\": \"$cfg\"}" >> gpurun_out/bb.jsonl
    RSORT_BUCKET_MW=$mw RSORT_BUCKET_SIGMA=$sig RSORT_BUCKET_PAD=$pad RSORT_BUCKET_WAVES=$wv timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 >> gpurun_out/bb.jsonl 2>> gpurun_out/bb.err || exit 11
  done
done
RSORT_BUCKET_MW=4 RSORT_BUCKET_SIGMA=4 RSORT_BUCKET_PAD=0 timeout -k 10 300 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bb_tests.log 2>&1 || exit 12
