set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -X faulthandler tools/range_time.py > gpurun_out/range_time.jsonl 2> gpurun_out/range_time.err || exit 11
