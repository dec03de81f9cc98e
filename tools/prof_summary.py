#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per-dispatch durations of the
transport kernel, the generation-0 launches (one per MC step, the large
ones) and their mean, to compare with bench.py's HIP-event kernel_ms_avg."""
import csv
import sys
from statistics import mean


def main(path, timed_last=None):
    rows = list(csv.DictReader(open(path)))
    tk = [r for r in rows if "transport_kernel" in r["Kernel_Name"]]
    tk.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in tk]
    # generation 0 = first launch of each step: the launches that follow a
    # non-transport dispatch gap; identify as durations > 1 ms
    g0 = [d for d in dur if d > 1.0]
    print("transport dispatches: %d" % len(dur))
    print("all durations (ms): %s" % ", ".join("%.3f" % d for d in dur))
    print("generation-0 launches: %d, durations (ms): %s" % (len(g0), ", ".join("%.3f" % d for d in g0)))
    if timed_last:
        sel = g0[-int(timed_last):]
        print("mean of the last %d generation-0 launches (bench timed steps): %.3f ms"
              % (len(sel), mean(sel)))
    r0 = tk[0]
    print("rocprofv3 fields (VGPR_Count is granule-encoded; tools/code_object.py prints the code "
          "object's register counts): VGPR=%s SGPR=%s LDS=%s scratch=%s workgroup=%s grid=%s" % (
        r0["VGPR_Count"], r0["SGPR_Count"], r0["LDS_Block_Size"], r0["Scratch_Size"],
        r0["Workgroup_Size_X"], r0["Grid_Size_X"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
