# Round 5: kernel stats of the presorted path (config 4, config3_check_order).
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/nsprof
for w in ${WL:-config4 config3_check_order}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nsprof/$w -o prof -- \
      python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/nsprof/$w.json 2> gpurun_out/nsprof/$w.log || { tail -20 gpurun_out/nsprof/$w.log; exit 1; }
done
find gpurun_out/nsprof -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 "$f" | head -30; done
exit 0
