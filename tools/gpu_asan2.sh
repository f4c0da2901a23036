# host ASan/UBSan/LSan driver over every C-ABI entry point (incl. the keys-only hybrid MSD path)
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ASAN_OPTIONS=halt_on_error=1 LSAN_OPTIONS=suppressions=tools/lsan.supp:print_suppressions=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 timeout -k 10 400 ./tools/asan_driver > gpurun_out/asan2.log 2>&1 || exit 13
