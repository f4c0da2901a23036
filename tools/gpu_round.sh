# One GPU call: full GPU test suite, smoke, bench lines, rocprof kernel stats and PMC traffic.
# Usage (GPU box, from the repo root): bash tools/gpu_round.sh [first_step]; results in gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
from=${1:-1}
step() { [ "$1" -ge "$from" ]; }
step 1 && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 10; }
step 2 && { timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 11; }
step 3 && { timeout -k 10 300 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit 12; }
step 4 && { timeout -k 10 300 python bench.py --workload config3_texture --no-cpu-baseline > gpurun_out/bench_tex.json 2> gpurun_out/bench_tex.err || exit 13; }
step 5 && { timeout -k 10 300 python bench.py --workload config2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 14; }
step 6 && { timeout -k 10 300 python -u bench.py --workload config4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 15; }
step 7 && { timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o b --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit 16; }
step 8 && { timeout -k 10 600 python3 tools/pmc_traffic.py config3 gpurun_out/traffic_c3.json > gpurun_out/pmc.log 2>&1 || exit 17; }
exit 0
