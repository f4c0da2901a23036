set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for lg in 21 22 23 24 25 26 28; do
  RSORT_TILE=large RSORT_ONESWEEP=1 timeout -k 10 120 python tools/mall_sort_probe.py $lg 20 >> gpurun_out/mall_sort_probe.jsonl 2>> gpurun_out/mall_sort_probe.err || exit 11
done
for lg in 22 23 24 28; do
  RSORT_TILE=large RSORT_ONESWEEP=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mall_$lg -o p --output-format csv -- python3 tools/mall_sort_probe.py $lg 20 >> gpurun_out/mall_sort_probe_prof.jsonl 2>> gpurun_out/mall_sort_probe.err || exit 12
done
