cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for r in 1 2; do
  for c in 1 3; do
    RSORT_MSD_KEYS_CFG=$c timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline --steps 20 > gpurun_out/ab_cfg${c}_r$r.json 2>/dev/null || exit 1
  done
done
