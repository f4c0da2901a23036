# keys-only bucket pass: waves per workgroup (RSORT_KWAVE_WPB) and the listed-bucket launch grid
# (RSORT_OVER_GRID), config2 bench; config3 with the smaller listed-bucket grid
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/kw.jsonl
for cfg in "X=1" "RSORT_KWAVE_WPB=2" "RSORT_KWAVE_WPB=8" "RSORT_OVER_GRID=32" "X=1" "RSORT_KWAVE_WPB=2" "RSORT_KWAVE_WPB=8" "RSORT_OVER_GRID=32"; do
  echo "{\"cfg\": \"$cfg\"}" >> gpurun_out/kw.jsonl
  env $cfg timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 >> gpurun_out/kw.jsonl 2>> gpurun_out/kw.err || exit 12
done
for cfg in "X=1" "RSORT_OVER_GRID=32"; do
  echo "{\"cfg\": \"$cfg\"}" >> gpurun_out/kw.jsonl
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 >> gpurun_out/kw.jsonl 2>> gpurun_out/kw.err || exit 13
done
RSORT_KWAVE_WPB=8 RSORT_OVER_GRID=32 timeout -k 10 400 python -u -m pytest tests/test_msd_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "keys" > gpurun_out/kw_tests.log 2>&1 || exit 11
