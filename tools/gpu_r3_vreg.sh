# round-3: the wide bucket kernel's variants (values re-read vs kept in registers) through the rank
# model (config-5 shape regions) and the single-GPU 2^29..2^31 sorts
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in vreg0 vreg1; do
  RSORT_LIB=$PWD/exp_lib/librsort_$v.so timeout -k 10 300 python -u tools/rank_model.py --reps 5 > gpurun_out/r3_rank_$v.json 2> gpurun_out/r3_rank_$v.err || exit 11
done
