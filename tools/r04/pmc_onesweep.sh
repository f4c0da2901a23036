# Round 4: SQ counters of the hybrid path's kernels on config3 (tools/prof_driver.py, 2 sorts), one
# rocprofv3 --pmc pass per counter group (each under its own SIGKILL limit), CSVs under gpurun_out/pmc_*.
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
pass() {   # pass <name> <counters...>
  local nm=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$nm -o p -- python3 tools/prof_driver.py config3 2 > gpurun_out/pmc_$nm.log 2>&1
  echo "pass $nm rc=$?" >> gpurun_out/pmc_status.txt
}
pass cycles SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass active SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS
pass insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES
exit 0
