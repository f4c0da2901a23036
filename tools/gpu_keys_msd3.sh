# keys-only bucket pass: wave kernel VGPR budget sweep (RSORT_KWAVE_MW), config2 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/km3_sweep.jsonl
for cfg in "RSORT_KWAVE_MW=1" "RSORT_KWAVE_MW=5" "RSORT_KWAVE_MW=6" "RSORT_KWAVE_MW=7" "RSORT_KWAVE_MW=1"; do
  echo "{\"cfg\": \"$cfg\"}" >> gpurun_out/km3_sweep.jsonl
  env $cfg timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 >> gpurun_out/km3_sweep.jsonl 2>> gpurun_out/km3.err || exit 12
done
RSORT_KWAVE_MW=6 timeout -k 10 400 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "keys and uniform" > gpurun_out/km3_tests.log 2>&1 || exit 11
