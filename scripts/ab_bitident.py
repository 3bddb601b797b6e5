"""Bit-identity check between two builds of libba3c.so (A/B of a layout-only change): run as
   BA3C_LIB=<lib> python scripts/ab_bitident.py dump OUT.npz   (each build, separate processes)
   python scripts/ab_bitident.py compare A.npz B.npz
dump: gradients, TfDictOp scalars and the workspace activations of one training pass at B=2048
(F=512, S=1), B=160 and B=32 (F=128, S=4) on fixed random frames."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-ba3c_amd"))
sys.path.insert(0, ROOT)


def dump(out):
    from ba3c_amd.engine import Ba3cEngine
    from oracle import ba3c_oracle as O
    res = {}
    for B, F, S in ((2048, 512, 1), (160, 512, 1), (32, 128, 4)):
        rs = np.random.RandomState(B)
        eng = Ba3cEngine(num_actions=4, fc_neurons=F, fc_splits=S, max_batch=B)
        eng.load_params(O.init_params(F, S, 4, seed=7, dtype=np.float32))
        st = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda()
        ac = torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda()
        R = torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()
        sc = eng.train_grads(st, ac, R)
        res["B%d_grads" % B] = eng.grads.cpu().numpy()
        res["B%d_scalars" % B] = sc.cpu().numpy()
        for n in ("p1", "p2", "dp1", "dp0"):
            res["B%d_%s" % (B, n)] = eng.workspace_tensor(n, B).cpu().numpy()
        torch.cuda.synchronize()
        assert eng.device_errors() == 0
        del eng
    np.savez(out, **res)


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k], Bz[k])]
    print("bit-identical: %d of %d arrays%s" % (len(A.files) - len(bad), len(A.files),
                                                 "; differ: %s" % bad if bad else ""))
    return 0 if not bad else 1


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
