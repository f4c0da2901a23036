# hybrid MSD path: checks, timing at two bucket slacks, LSD timing, rocprof kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RSORT_MSD=1 timeout -k 10 400 python tools/msd_check.py check > gpurun_out/msd_check.jsonl 2> gpurun_out/msd_check.err || exit 11
RSORT_MSD=1 timeout -k 10 200 python tools/msd_check.py time > gpurun_out/msd_time.jsonl 2>> gpurun_out/msd_check.err || exit 12
RSORT_MSD=1 RSORT_BUCKET_SLACK=1.15 timeout -k 10 200 python tools/msd_check.py time >> gpurun_out/msd_time.jsonl 2>> gpurun_out/msd_check.err || exit 13
RSORT_MSD=0 timeout -k 10 200 python tools/msd_check.py time >> gpurun_out/msd_time.jsonl 2>> gpurun_out/msd_check.err || exit 14
RSORT_MSD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_msd -o m --output-format csv -- python3 tools/msd_check.py time > gpurun_out/msd_prof.jsonl 2>> gpurun_out/msd_check.err || exit 15
