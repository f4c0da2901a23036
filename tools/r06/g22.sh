# Round 6: address-translation counters of the MSD passes (is pass 0's scattered write pattern a TLB cost?)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/tlb
[ -f gpurun_out/tlb/avail.txt ] && grep -o -E "\b(TCP_UTCL1[A-Z0-9_]*|UTCL2[A-Z0-9_]*|TCP_TCP_TA_DATA_STALL[A-Z_]*|TCP_PENDING_STALL[A-Z_]*|TCP_TCR_TCP_STALL[A-Z_]*|TCP_WRITE_TAGCONFLICT_STALL[A-Z_]*|TCP_READ_TAGCONFLICT_STALL[A-Z_]*|TA_ADDR_STALLED_BY_TC_CYCLES[A-Z_]*|TA_DATA_STALLED_BY_TC_CYCLES[A-Z_]*)\b" gpurun_out/tlb/avail.txt | sort -u > gpurun_out/tlb/names.txt
cat gpurun_out/tlb/names.txt | tr '\n' ' '; echo
run() {  # one --pmc pass (at most 4 TCP_ / 2 TA_ counters)
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/tlb/$1 -o p -- python3 tools/prof_driver.py config3 2 > gpurun_out/tlb/$1.log 2>&1
}
sum() { python3 - "$1" <<'PY'
import csv,glob,sys
acc={}
for f in glob.glob(f"gpurun_out/tlb/{sys.argv[1]}/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        n=r["Kernel_Name"]
        k="pass0" if "k_msd_pass<1" in n else "pass1" if "k_msd_pass<2" in n else "bucket" if "k_bucket_sort<256" in n else "hist16" if "k_hist16_in" in n else None
        if k:
            e=acc.setdefault((k,r["Counter_Name"]),[0.0,set()]); e[0]+=float(r["Counter_Value"]); e[1].add(r.get("Dispatch_Id",""))
for (k,c),(v,d) in sorted(acc.items()): print(k,c,round(v/max(1,len(d))))
PY
}
run TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_REQUEST TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS && sum TCP_UTCL1_TRANSLATION_MISS
run TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES && sum TA_ADDR_STALLED_BY_TC_CYCLES
run TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_WRITE_TAGCONFLICT_STALL_CYCLES TCP_UTCL1_THRASHING_STALL && sum TCP_PENDING_STALL_CYCLES
exit 0
