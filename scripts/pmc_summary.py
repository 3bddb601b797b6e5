"""Per-kernel averages of rocprofv3 --pmc passes (counter_collection.csv files).

usage: pmc_summary.py DIR [--json OUT]   (DIR holds pmc*/run_counter_collection.csv)

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB.  HBM bytes per launch
follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced read, so it is doubled; WRITE_SIZE is taken as is."""
import collections
import csv
import glob
import json
import os
import re
import sys

SHORT = [  # (regex on the kernel symbol, bench kernel id)
    (r"conv0s_fwd_kernel|conv0_band_kernel", "conv0_fwd"),
    (r"conv0s_wgrad_kernel|wgrad01_pair_kernel", "conv0_wgrad"),
    (r"conv_band6[rp]?_kernel<.*BandGeom<40, 40, 32, 32", "conv1_fwd"),
    (r"conv_band6[rp]?_kernel<.*BandGeom<18, 18, 32, 64", "conv2_fwd"),
    (r"(conv_band6[rp]?_kernel|multi_kernel_w2)<.*BandGeom<44, 44, 32, 32", "conv1_dgrad"),
    (r"(conv_band6[rp]?_kernel|multi_kernel_w2)<.*BandGeom<22, 22, 64, 32", "conv2_dgrad"),
    (r"wgrad6?w?_(band_)?kernel<.*Geom<40, 40, 32", "conv1_wgrad"),
    (r"wgrad6?_(band_)?kernel<.*Geom<18, 18, 32", "conv2_wgrad"),
    (r"conv3_band_kernel<false>|ConvFwd<false, 7, 7, 64", "conv3_fwd"),
    (r"conv3_band_kernel<true>|Conv3DJob|ConvDgrad<7, 7, 64", "conv3_dgrad"),
    (r"conv3_wgrad_kernel|ConvWgrad<false, 7, 7, 64", "conv3_wgrad"),
    (r"FcFwd", "fc1_fwd"), (r"FcDgrad", "fc1_dgrad"),
    (r"gemm6?_kernel<128, 64, 2, 2, ba3c::BatchWgrad", "fc1_wgrad"),
    (r"gemm6?_kernel<128, 32, 4, 1, ba3c::BatchWgrad", "head_wgrad"),
    (r"heads_kernel", "heads"), (r"wgrad_reduce(_all)?_kernel", "wgrad_reduce"),
    (r"update_kernel", "update"), (r"sumsq_kernel", "sumsq"),
    (r"wprep6?_kernel", "wprep"), (r"scalars_kernel", "scalars"),
]


def short(name):
    for rx, k in SHORT:
        if re.search(rx, name):
            return k
    return None


def load(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        per = collections.defaultdict(float)   # (dispatch, counter) -> summed over dims
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (disp, ctr), v in per.items():
            k = short(names[disp])
            if k:
                acc[k][ctr].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    d = sys.argv[1]
    res = load(d)
    for k, cs in res.items():
        if "FETCH_SIZE" in cs or "WRITE_SIZE" in cs:
            cs["hbm_bytes"] = 2.0 * cs.get("FETCH_SIZE", 0.0) * 1024 + cs.get("WRITE_SIZE", 0.0) * 1024
    if "--json" in sys.argv:
        src = sys.argv[sys.argv.index("--source") + 1] if "--source" in sys.argv else d
        doc = {"source": src,
               "hbm_bytes": "per launch: 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024); FETCH_SIZE "
                            "doubled per MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B "
                            "requests at 64 B); one --pmc pass per counter group",
               "kernels": res}
        json.dump(doc, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1, sort_keys=True)
    cols = ["hbm_bytes", "FETCH_SIZE", "WRITE_SIZE", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE",
            "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
            "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS", "SQ_LDS_UNALIGNED_STALL", "SQ_WAVE_CYCLES",
            "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"]
    extra = sorted({c for cs in res.values() for c in cs} - set(cols))
    cols = [c for c in cols if any(c in cs for cs in res.values())] + extra
    print("| kernel | " + " | ".join(cols) + " |")
    print("|---" * (len(cols) + 1) + "|")
    for k in sorted(res):
        cs = res[k]
        print("| %s | " % k + " | ".join("%.4g" % cs[c] if c in cs else "-" for c in cols) + " |")


if __name__ == "__main__":
    main()
