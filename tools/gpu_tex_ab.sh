# texture-layout histogram A/B: the previous commit's library vs the current one, alternated
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for lib in old new old new; do
  if [ $lib = old ]; then L=webgpu-radix-sort_amd/lib/librsort_old.so; else L=webgpu-radix-sort_amd/lib/librsort.so; fi
  echo "{\"lib\": \"$lib\"}" >> gpurun_out/ab.jsonl
  RSORT_LIB=$PWD/$L timeout -k 10 200 python bench.py --workload config3_texture --no-cpu-baseline --steps 20 >> gpurun_out/ab.jsonl 2>> gpurun_out/ab.err || exit 12
done
