"""Kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage remarks.
usage: make -C distributed-ba3c_amd resource-usage 2>&1 | python scripts/resource_table.py [filter]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0].replace("\\", "")] = int(m.group(1))
print("| kernel | VGPR | AGPR | scratch | waves/SIMD | LDS |")
print("|---|---|---|---|---|---|")
for r in rows:
    n = r["name"].replace("void ba3c::", "").replace("ba3c::", "")
    if flt and flt not in n:
        continue
    n = re.sub(r"\(.*\)$", "", n)[:120]
    print("| %s | %s | %s | %s | %s | %s |" % (n, r.get("VGPRs"), r.get("AGPRs"), r.get("ScratchSize"),
                                              r.get("Occupancy"), r.get("LDS")))
