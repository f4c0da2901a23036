# tuning sweep over lib/variants (tools/sweep.py); args = variant specs (name[@ENV=v...])
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python tools/sweep.py "$@" > gpurun_out/sweep.jsonl 2> gpurun_out/sweep.err
