"""Turn a rocprofv3 run (rocpd SQLite db, or its kernels_summary.csv) into the markdown
kernel table kept under profiles/.  usage: prof_summary.py RUN_RESULTS.db|SUMMARY.csv [TITLE]"""
import csv
import os
import subprocess
import sys
import tempfile


def summary_csv(path):
    if path.endswith(".csv"):
        return path
    out = tempfile.mkdtemp(prefix="rocpd_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    subprocess.check_call(["/opt/rocm/bin/rocpd2summary", "-i", os.path.abspath(path), "-f", "csv",
                           "-d", out, "-o", "run"], cwd="/tmp", env=env,
                          stdout=subprocess.DEVNULL)
    return os.path.join(out, "run_kernels_summary.csv")


def short(name):
    name = name.replace("void ", "").replace("ba3c::", "")
    return name[:110]


def main():
    rows = list(csv.DictReader(open(summary_csv(sys.argv[1]))))
    for r in rows:   # rocpd2summary vs rocprofv3 --output-format csv column names
        r.setdefault("Duration (Nsec)", r.get("TotalDurationNs"))
        r.setdefault("Average (Nsec)", r.get("AverageNs"))
    total = sum(float(r["Duration (Nsec)"]) for r in rows)
    title = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(sys.argv[1])
    print("# %s\n" % title)
    print("| kernel | calls | avg µs | total ms | % |")
    print("|---|---|---|---|---|")
    for r in rows:
        d = float(r["Duration (Nsec)"])
        print("| `%s` | %s | %.1f | %.2f | %.2f |" % (short(r["Name"]), r["Calls"],
              float(r["Average (Nsec)"]) / 1e3, d / 1e6, 100.0 * d / total))


if __name__ == "__main__":
    main()
