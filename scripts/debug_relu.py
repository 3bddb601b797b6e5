"""active_relus of one train step (GPU) against the oracle's per-layer counts (debug)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "distributed-ba3c_amd"); sys.path.insert(0, ".")
from oracle import ba3c_oracle as O
from ba3c_amd.engine import Ba3cEngine
B = 160
rs = np.random.RandomState(3)
params = O.init_params(512, 1, 4, seed=7)
params = {k: (v * 2).astype(np.float32) for k, v in params.items()}
state = rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)
a = rs.randint(0, 4, size=B).astype(np.int64); R = rs.normal(size=B).astype(np.float32)
eng = Ba3cEngine(num_actions=4, fc_neurons=512, fc_splits=1, max_batch=B)
eng.load_params(params)
d = lambda x: torch.from_numpy(x).cuda()
sc = eng.train_grads(d(state), d(a), d(R)).cpu().numpy()
cnt = [0, 0, 0, 0]
for lo in range(0, B, 16):
    t = O.get_nn_prediction({k: v.astype(np.float64) for k, v in params.items()}, state[lo:lo + 16], {"fc_neurons": 512, "fc_splits": 1})
    for l in range(4):
        cnt[l] += int(np.count_nonzero(t["a%d" % l]))
print("gpu", int(sc[7]), "oracle", sum(cnt), cnt)
