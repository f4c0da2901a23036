# rocprofv3 kernel stats of bench.py (config3) with and without the 24K-record tiles.
# Usage (GPU box): bash tools/prof_kernels.sh  -> gpurun_out/prof_{huge,base}/...stats.csv
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_huge -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/prof_huge.json 2> gpurun_out/prof_huge.err || exit 11
RSORT_HUGE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base -o p --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/prof_base.json 2> gpurun_out/prof_base.err || exit 12
