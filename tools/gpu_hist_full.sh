# 16-bit histogram specialised for the whole key range vs the generic range-relative counting
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_msd_gpu.py tests/test_texture_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/hf_tests.log 2>&1 || exit 11
: > gpurun_out/hf.jsonl
for wl in config3 config3_texture config2; do
for cfg in "X=1" "RSORT_HIST16_GENERIC=1" "X=1" "RSORT_HIST16_GENERIC=1"; do
  echo "{\"cfg\": \"$cfg\"}" >> gpurun_out/hf.jsonl
  env $cfg timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline --steps 20 >> gpurun_out/hf.jsonl 2>> gpurun_out/hf.err || exit 12
done
done
