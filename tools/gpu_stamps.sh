# k_onesweep phase stamps + config3 bench per prefetch/ticket variant (diagnostic builds)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for v in s_pf0 s_pf1 s_pf2 s_pf1et s_pf0et; do
  export RSORT_LIB=webgpu-radix-sort_amd/lib/variants/librsort_$v.so
  echo "== $v" >> gpurun_out/stamps.jsonl
  timeout -k 10 120 python tools/stamp_probe.py 28 >> gpurun_out/stamps.jsonl 2>> gpurun_out/stamps.err || exit 11
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/bench_$v.json 2>> gpurun_out/stamps.err || exit 12
  echo "$v $(cut -c1-330 gpurun_out/bench_$v.json)" >> gpurun_out/stamps_bench.txt
done
