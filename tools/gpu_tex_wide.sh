# texture-layout 16-bit histogram: two records per 16-byte load vs one per 8-byte load
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_msd_gpu.py tests/test_texture_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tw_tests.log 2>&1 || exit 11
: > gpurun_out/tw.jsonl
for cfg in "X=1" "RSORT_HIST16_NARROW=1" "X=1" "RSORT_HIST16_NARROW=1"; do
  echo "{\"cfg\": \"$cfg\"}" >> gpurun_out/tw.jsonl
  env $cfg timeout -k 10 200 python bench.py --workload config3_texture --no-cpu-baseline --steps 20 >> gpurun_out/tw.jsonl 2>> gpurun_out/tw.err || exit 12
done
