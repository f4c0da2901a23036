# Round 4: SQ counters of the single-pass scan (k_scan_lookback, 2^28 u32; tools/prof_driver.py
# prefix_sum, 2 launches), one rocprofv3 --pmc pass per counter group (each under its own SIGKILL
# limit), CSVs under gpurun_out/pmc_scan_*.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
pass() {   # pass <name> <counters...>
  local nm=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_scan_$nm -o p -- python3 tools/prof_driver.py prefix_sum 2 > gpurun_out/pmc_scan_$nm.log 2>&1
  echo "pass $nm rc=$?" >> gpurun_out/pmc_status.txt
}
pass cycles SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass active SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS
exit 0
