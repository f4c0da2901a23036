# keys-only hybrid MSD path, round 2: parity tests, config2 bench variants
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k keys > gpurun_out/km2_tests.log 2>&1 || exit 11
: > gpurun_out/km2_sweep.jsonl
for cfg in "X=1" "RSORT_KBUCKET_WAVE=0" "RSORT_KBUCKET_WAVE=0 RSORT_KBUCKET_PF=0" "RSORT_MSD=0" "X=2"; do
  echo "{\"cfg\": \"$cfg\"}" >> gpurun_out/km2_sweep.jsonl
  env $cfg timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 >> gpurun_out/km2_sweep.jsonl 2>> gpurun_out/km2.err || exit 12
done
