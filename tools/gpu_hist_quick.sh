set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hq -o h --output-format csv -- python3 tools/msd_check.py time > gpurun_out/hq.jsonl 2> gpurun_out/hq.err || exit 11
