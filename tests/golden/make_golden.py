"""Generate the committed golden fixtures under tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`).

* fwd_B4_C4.npz, fwd_B3_C12.npz  — predictor outputs of the float64 oracle on fixed frames
* step_B8_F128_S4.npz            — raw gradients + TfDictOp scalars of one tower, and the
                                   parameters after one clip + TF-Adam apply (beta1 0.8,
                                   beta2 0.75, eps 1e-8, lr 1e-3: README best run)
* sample_A4.npz, sample_A18.npz  — action draws of numpy's own RandomState.choice (the
                                   reference's train.py:382 call): pinned to the library,
                                   not to the oracle

Weights are regenerated from their seed by oracle.init_params (legacy numpy RandomState, a
stable stream), so the fixtures hold only inputs the seed does not determine and outputs.
The network fixtures are "parity unpinned" (no reference run is possible here).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import ba3c_oracle as O  # noqa: E402


def _params(F, S, A, seed):
    p = O.init_params(F, S, A, seed=seed, dtype=np.float32)
    return {k: v.astype(np.float64) for k, v in p.items()}, p


def fwd(name, B, C, F, S, A, seed, explore):
    p64, _ = _params(F, S, A, seed)
    rs = np.random.RandomState(seed + 1)
    state = rs.randint(0, 256, size=(B, 84, 84, C)).astype(np.uint8)
    t = O.get_nn_prediction(p64, state, {"fc_neurons": F, "fc_splits": S}, explore_factor=explore)
    np.savez_compressed(os.path.join(HERE, name), seed=seed, F=F, S=S, A=A, C=C, explore=explore,
                        state=state, logits=t["logits"], logitsT=t["logitsT"],
                        pred_value=t["pred_value"], h=t["h"])


def step(name, B, F, S, A, seed):
    p64, p32 = _params(F, S, A, seed)
    rs = np.random.RandomState(seed + 1)
    state = rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)
    action = rs.randint(0, A, size=B).astype(np.int64)
    R = rs.normal(size=B).astype(np.float32)
    cfg = {"fc_neurons": F, "fc_splits": S}
    _, sc, g = O.loss_and_grads(p64, state, action, R.astype(np.float64), cfg)
    slots = O.init_slots(p64, "adam", 0.8, 0.75)
    newp, _, _, _ = O.train_step(p64, slots, 1, [(state, action, R.astype(np.float64))], cfg,
                                 lr=1e-3, beta1=0.8, beta2=0.75, eps=1e-8)
    out = dict(seed=seed, F=F, S=S, A=A, state=state, action=action, R=R)
    for k, v in g.items():   # float32 storage: checked at 1e-4 relative
        out["grad:" + k] = v.astype(np.float32)
        out["adam1_delta:" + k] = (newp[k] - p64[k]).astype(np.float32)
    for k, v in sc.items():
        out["scalar:" + k] = np.float64(v)
    np.savez_compressed(os.path.join(HERE, name), **out)


def sample(name, A, n, seed):
    rs = np.random.RandomState(seed)
    probs = rs.dirichlet(np.ones(A) * 0.5, size=n).astype(np.float32)
    probs[::17] = 0
    probs[::17, 0] = 1.0
    actions = O.np_random_choice(probs, np.random.RandomState(seed + 1000))
    u = O.draw_uniforms(n, np.random.RandomState(seed + 1000))
    np.savez_compressed(os.path.join(HERE, name), probs=probs, u=u, actions=actions,
                        rng_seed=seed + 1000)


if __name__ == "__main__":
    fwd("fwd_B4_C4.npz", 4, 4, 128, 4, 4, seed=7, explore=1.0)
    fwd("fwd_B3_C12.npz", 3, 12, 256, 2, 6, seed=8, explore=1.5)
    step("step_B8_F128_S4.npz", 8, 128, 4, 4, seed=9)
    sample("sample_A4.npz", 4, 4000, seed=10)
    sample("sample_A18.npz", 18, 2000, seed=11)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
