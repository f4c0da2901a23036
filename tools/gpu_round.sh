# One GPU call: full GPU test suite, smoke, bench lines, rocprof kernel stats and PMC traffic.
# Usage (GPU box, from the repo root): bash tools/gpu_round.sh [first_step [last_step]]; results in
# gpurun_out/.  Every step has its own time limit; the first failure ends the call.
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
from=${1:-1}
to=${2:-99}
step() { [ "$1" -ge "$from" ] && [ "$1" -le "$to" ]; }
bench() {   # bench <step> <workload> <extra args...>
    local n=$1 w=$2; shift 2
    timeout -k 10 300 python -u bench.py --workload "$w" "$@" > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || exit $((10 + n))
}
step 1 && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 11; }
step 2 && { timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 12; }
step 3 && { timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 13; }
step 4 && bench 4 config3_texture --no-cpu-baseline
step 5 && bench 5 config2 --no-cpu-baseline
step 6 && bench 6 config4 --no-cpu-baseline
step 7 && bench 7 config3_check_order --no-cpu-baseline
step 8 && { timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o b --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit 18; }
step 9 && { for w in config3 config2 config4; do timeout -k 10 600 python3 tools/pmc_traffic.py $w gpurun_out/traffic_$w.json > gpurun_out/pmc_$w.log 2>&1 || exit 19; done; }
step 10 && { timeout -k 10 600 python3 -u tools/rank_model.py > gpurun_out/rank_model.json 2> gpurun_out/rank_model.err || exit 20; }
# the driver's N-GPU bench path (plain --gpus N -> torch.distributed.run -> N ranks) rehearsed with
# 2 ranks sharing GPU 0 over gloo (host-staged exchange: not a measurement)
step 11 && { timeout -k 10 400 python3 bench.py --gpus 2 --share-gpu --keys-per-gpu 67108864 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_rehearsal_2ranks.json 2> gpurun_out/bench_rehearsal_2ranks.err || exit 21; }
# host ASan/UBSan/LSan driver over every C-ABI entry point (built here: make -C
# webgpu-radix-sort_amd/csrc asan; the binary and the asan library must not be gpurun-ignored
# for this step)
step 12 && { ASAN_OPTIONS=halt_on_error=1 LSAN_OPTIONS=suppressions=tools/lsan.supp:print_suppressions=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 timeout -k 10 400 ./tools/asan_driver > gpurun_out/asan_driver.log 2>&1 || exit 22; }
# SQ / TCC counters per kernel (config 3 and a multi-GPU receiver's regions), one --pmc pass per group
step 13 && { for w in config3 region; do timeout -k 10 600 python3 tools/pmc_sq.py $w gpurun_out/pmc_sq_$w > gpurun_out/pmc_sq_$w.log 2>&1 || exit 23; done; }
exit 0
