"""Kernel durations of the forward kernels in a training step vs a predictor forward (no argmax
codes, no ReLU counts) at B=2048: run under rocprofv3 --kernel-trace, then
`python scripts/fwd_vs_train.py --report DIR/run_kernel_trace.csv`."""
import csv
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "distributed-ba3c_amd")]


def run():
    import numpy as np
    import torch
    from ba3c_amd.engine import Ba3cEngine
    torch.cuda.set_device(0)
    B = 2048
    eng = Ba3cEngine(num_actions=4, fc_neurons=512, fc_splits=1, max_batch=B)
    eng.init_params(seed=0)
    g = torch.Generator(device="cuda").manual_seed(0)
    st = torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device="cuda", generator=g)
    ac = torch.randint(0, 4, (B,), dtype=torch.int64, device="cuda", generator=g)
    R = torch.randn(B, dtype=torch.float32, device="cuda", generator=g)
    for _ in range(6):
        eng.train_grads(st, ac, R)
    torch.cuda.synchronize()
    for _ in range(6):
        eng.forward(st)
    torch.cuda.synchronize()
    print("done")


def report(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "ba3c" in r["Kernel_Name"]]
    seq = []
    for r in rows:
        n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("ba3c::", "")[:60]
        seq.append((n, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    half = len(seq) // 2
    for tag, part in (("train", seq[:half]), ("forward", seq[half:])):
        acc = {}
        for n, d in part[len(part) // 3:]:
            acc.setdefault(n, []).append(d)
        print(tag)
        for n, v in acc.items():
            print("  %-60s %8.1f us (%d)" % (n, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
