"""Per-step kernel timeline from a rocprofv3 kernel trace: start / end / duration relative to the
step's first kernel (wprep6), queue, grid, and the idle gaps of the main queue.

usage: step_timeline.py run_kernel_trace.csv [step index]"""
import csv
import re
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    idx = [i for i, r in enumerate(rows) if re.search(r"wprep6|WPrep6Job", r["Kernel_Name"])]
    s, e = idx[k], idx[k + 1]
    t0 = int(rows[s]["Start_Timestamp"])
    busy = 0
    for r in rows[s:e]:
        st, en = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        wg = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // int(r["Workgroup_Size_X"])
        busy += en - st
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("ba3c::", "")[:90]
        print("%7.1f %7.1f %6.1f q%s wg=%-5d %s" % (st / 1e3, en / 1e3, (en - st) / 1e3, r["Queue_Id"], wg, name))
    print("step %.1f us, %d kernels, summed durations %.1f us"
          % ((int(rows[e]["Start_Timestamp"]) - t0) / 1e3, e - s, busy / 1e3))


if __name__ == "__main__":
    main()
