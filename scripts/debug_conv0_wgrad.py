"""Diagnostic: conv0/W gradient of the band path vs the generic path vs the fp32 oracle over
batch sizes (test infrastructure; imports the oracle as the checker)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-ba3c_amd"))
from oracle import ba3c_oracle as O  # noqa: E402


def engine(generic):
    os.environ["BA3C_GENERIC"] = "1" if generic else "0"
    from ba3c_amd.engine import Ba3cEngine
    e = Ba3cEngine(num_actions=4, channels=4, fc_neurons=128, fc_splits=4, max_batch=64)
    os.environ.pop("BA3C_GENERIC")
    return e


def main():
    p32 = O.init_params(128, 4, 4, seed=9, dtype=np.float32)
    cfg = {"fc_neurons": 128, "fc_splits": 4}
    eb, eg = engine(False), engine(True)
    for e in (eb, eg):
        e.load_params(p32)
    cases = [(8, 10), (8, 10)] + [(B, B) for B in (1, 5, 8, 9, 16, 33)]
    for B, seed in cases:
        rs = np.random.RandomState(seed)
        s = rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)
        a = rs.randint(0, 4, size=B).astype(np.int64)
        r = rs.normal(size=B).astype(np.float32)
        _, _, g = O.loss_and_grads(p32, s, a, r, cfg)
        line = ["B=%2d" % B]
        for tag, e in (("band", eb), ("gen", eg)):
            e.train_grads(torch.from_numpy(s).cuda(), torch.from_numpy(a).cuda(), torch.from_numpy(r).cuda())
            got = e.state_dict(e.grads)
            worst = max(g, key=lambda k: np.abs(got[k] - g[k]).max() / np.abs(g[k]).max())
            line.append("%s worst %s %.2e" % (tag, worst, np.abs(got[worst] - g[worst]).max() / np.abs(g[worst]).max()))
            t, _, _ = O.loss_and_grads(p32, s, a, r, cfg)
            flips = []
            shapes = {0: (B, 40, 40, 32), 1: (B, 18, 18, 32), 2: (B, 7, 7, 64)}
            for L in range(3):
                c = e.workspace_tensor("c%d" % L, B).cpu().numpy().reshape(shapes[L])
                own = np.where(t["p%d" % L] > 0, t["c%d" % L], 255)
                flips.append(int((own != c).sum()))
                p = e.workspace_tensor("p%d" % L, B).cpu().numpy().reshape(shapes[L])
                flips.append("%.1e" % (np.abs(p - t["p%d" % L]).max() / np.abs(t["p%d" % L]).max()))
            line.append("flips/perr %s" % (flips,))
            if tag == "band":
                gb = got
        line.append("band-vs-gen conv0 %.2e" % (np.abs(gb["conv0/W"] - got["conv0/W"]).max() / np.abs(got["conv0/W"]).max()))
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
