"""Kernel timeline of a rocprofv3 kernel trace (tools/r06_slot_trace2.sh): start, duration, queue, grid, name."""
import csv, sys
ls = sys.argv[1]
rows = sorted(csv.DictReader(open("/tmp/slot_ls%s/run_kernel_trace.csv" % ls)), key=lambda r: int(r["Start_Timestamp"]))
t0 = None
out = open("gpurun_out/r06s_timeline_full_ls%s.txt" % ls, "w")
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t0 = t0 or s
    out.write("%10.1f %10.1f us  q%s grid %s  %s\n" % ((s - t0) / 1e3, (e - s) / 1e3, r["Queue_Id"], r["Grid_Size_X"], r["Kernel_Name"][:40]))
