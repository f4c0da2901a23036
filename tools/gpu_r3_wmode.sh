# round-3: wide-bucket variants (sweep library): RSORT_WIDE_MODE 0 (product), 1 (values in
# registers), 2 (8-byte staging 256 x 34 for <= 8704-record buckets)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in 0 1 2; do
  RSORT_WIDE_MODE=$m RSORT_LIB=$PWD/exp_lib/librsort_wmode.so timeout -k 10 300 python -u tools/rank_model.py --reps 5 > gpurun_out/r3_wmode$m.json 2> gpurun_out/r3_wmode$m.err || exit 11
done
