# hybrid MSD path: parity/property checks with RSORT_MSD=1, then config3 timing on / off
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RSORT_MSD=1 timeout -k 10 400 python tools/msd_check.py check > gpurun_out/msd_check.jsonl 2> gpurun_out/msd_check.err || exit 11
RSORT_MSD=1 timeout -k 10 200 python tools/msd_check.py time > gpurun_out/msd_time.jsonl 2>> gpurun_out/msd_check.err || exit 12
RSORT_MSD=0 timeout -k 10 200 python tools/msd_check.py time >> gpurun_out/msd_time.jsonl 2>> gpurun_out/msd_check.err || exit 13
