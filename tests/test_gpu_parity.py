"""HIP path (through the C ABI) vs the CPU oracle on identical weights and inputs.

Tolerances (north star, BASELINE.json): forward logits/values within 1e-5 relative; gradients
and one optimizer step within 1e-4 relative; action sampling bit-exact given identical (p, u).
Relative error of a tensor = max|gpu - ref| / max|ref| (per tensor, avoids near-zero blowup).
"""
import numpy as np
import pytest
import torch

from oracle import ba3c_oracle as O

pytestmark = pytest.mark.gpu

FWD_TOL = 1e-5
GRAD_TOL = 1e-4

_ENGINES = {}


def engine(A=4, C=4, F=128, S=4, legacy=False, ps=1, max_batch=64, generic=False):
    """generic=True selects the gathered-tile GEMM engine for every conv (BA3C_GENERIC=1)
    instead of the LDS band kernels, so both code paths are held to the oracle."""
    import os
    from ba3c_amd.engine import Ba3cEngine
    key = (A, C, F, S, legacy, ps, max_batch, generic)
    if key not in _ENGINES:
        old = os.environ.get("BA3C_GENERIC")
        os.environ["BA3C_GENERIC"] = "1" if generic else "0"
        try:
            _ENGINES[key] = Ba3cEngine(num_actions=A, channels=C, fc_neurons=F, fc_splits=S,
                                       replace_with_conv=not legacy, ps=ps, max_batch=max_batch)
        finally:
            if old is None:
                del os.environ["BA3C_GENERIC"]
            else:
                os.environ["BA3C_GENERIC"] = old
    return _ENGINES[key]


def case(seed, B, A=4, C=4, F=128, S=4, legacy=False, ps=1, wscale=1.0, generic=False):
    rs = np.random.RandomState(seed)
    params = O.init_params(F, S, A, seed=seed, replace_with_conv=not legacy, ps=ps,
                           dtype=np.float32)
    for k in params:
        params[k] = (params[k] * np.float32(wscale)).astype(np.float32)
    state = rs.randint(0, 256, size=(B, 84, 84, C)).astype(np.uint8)
    action = rs.randint(0, A, size=B).astype(np.int64)
    R = rs.normal(size=B).astype(np.float32)
    cfg = {"fc_neurons": F, "fc_splits": S, "replace_with_conv": not legacy, "ps": ps}
    return params, state, action, R, cfg


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.abs(b).max()
    return float(np.abs(a - b).max() / den) if den > 0 else float(np.abs(a - b).max())


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def as64(params):
    return {k: v.astype(np.float64) for k, v in params.items()}


def gpu_decisions(eng, B):
    """The HIP path's own max-pool argmax codes and conv3 ReLU mask of the last train call."""
    shapes = {0: (B, 40, 40, 32), 1: (B, 18, 18, 32), 2: (B, 7, 7, 64)}
    codes = [eng.workspace_tensor("c%d" % l, B).cpu().numpy().reshape(shapes[l]) for l in range(3)]
    a3 = eng.workspace_tensor("a3", B).cpu().numpy().reshape(B, 5, 5, 64)
    forced = {"c0": codes[0], "c1": codes[1], "c2": codes[2], "a3_mask": a3 > 0}
    return forced, codes


def value_err(v_gpu, t, params):
    """|dV| relative to the magnitude of the summed terms of V = h.Wv + b (normwise: an fp32
    evaluation of a sum with cancellation is only accurate to eps * sum|terms|)."""
    scale = (np.abs(t["h"]) @ np.abs(params["fc-v/W"].astype(np.float64)))[:, 0] + abs(float(params["fc-v/b"][0]))
    return float(np.abs(np.asarray(v_gpu, np.float64) - t["pred_value"]).max() / scale.max())


CONFIGS = [
    dict(A=4, C=4, F=128, S=4),                 # BASELINE cfg2 geometry
    dict(A=6, C=12, F=512, S=1),                # RGB x4 frames, default F
    dict(A=18, C=4, F=256, S=1, legacy=True, ps=4),   # --use_normal_fc legacy FC
    dict(A=4, C=4, F=512, S=1, generic=True),   # gathered-tile GEMM engine for every conv
]


@pytest.mark.parametrize("cfgk", CONFIGS)
@pytest.mark.parametrize("B", [1, 7, 32])
def test_forward_matches_oracle(cfgk, B):
    params, state, _, _, cfg = case(11 + B, B, **cfgk)
    eng = engine(**cfgk)
    eng.load_params(params)
    probs, probsT, value = eng.forward(dev(state), explore_factor=1.7)
    t = O.get_nn_prediction(as64(params), state, cfg, explore_factor=1.7)
    torch.cuda.synchronize()
    assert rel(probs.cpu().numpy(), t["logits"]) < FWD_TOL
    assert rel(probsT.cpu().numpy(), t["logitsT"]) < FWD_TOL
    assert value_err(value.cpu().numpy(), t, params) < FWD_TOL


@pytest.mark.parametrize("cfgk", CONFIGS)
@pytest.mark.parametrize("B", [5, 32])
def test_gradients_and_scalars_match_oracle(cfgk, B):
    params, state, action, R, cfg = case(100 + B, B, wscale=2.0, **cfgk)
    eng = engine(**cfgk)
    eng.load_params(params)
    sc = eng.train_grads(dev(state), dev(action), dev(R), entropy_beta=0.01)
    got = eng.state_dict(eng.grads)
    forced, codes = gpu_decisions(eng, B)
    t, osc, g = O.loss_and_grads(as64(params), state, action, R.astype(np.float64), cfg,
                                 forced=forced)
    # discrete decisions (first-max argmax, ReLU sign) may differ only on fp32 near-ties
    for layer in range(3):
        own = np.where(t["p%d" % layer] > 0, t["c%d" % layer], 255)
        assert np.mean(own != codes[layer]) < 1e-4, layer
    assert np.mean((t["a3"] > 0) != forced["a3_mask"]) < 1e-4
    for k in g:
        e = rel(got[k], g[k])
        assert e < GRAD_TOL, (k, e)
    # padded conv0 input channels carry exactly zero gradient
    assert np.all(got["conv0/W"][:, :, cfgk["C"]:, :] == 0)
    s = sc.cpu().numpy()
    from ba3c_amd._lib import SCALAR_NAMES
    for i, name in enumerate(SCALAR_NAMES):
        ref = float(osc[name])
        assert abs(s[i] - ref) <= 1e-4 * max(1.0, abs(ref)), (name, s[i], ref)
    # count_nonzero of ReLU outputs: a pre-activation within fp32 rounding of 0 may flip
    assert abs(int(s[7]) - osc["active_relus"]) <= max(2, 1e-5 * osc["active_relus"])


def test_clip_kernel_matches_tf_formula():
    params, state, action, R, cfg = case(7, 16, wscale=2.0)
    eng = engine()
    eng.load_params(params)
    eng.train_grads(dev(state), dev(action), dev(R))
    raw = eng.state_dict(eng.grads)
    eng.clip_grads()
    clipped = eng.state_dict(eng.grads)
    for k in raw:
        ref = O.clip_by_average_norm(raw[k])
        assert rel(clipped[k], ref) < 2e-6, k


@pytest.mark.parametrize("opt", ["adam", "rms", "gd", "momentum", "adagrad", "adadelta"])
def test_optimizer_kernel_matches_tf_functor(opt):
    """Same gradient in, float32 TF-1.2 functor arithmetic out (3 consecutive applies)."""
    from ba3c_amd.optimizer import make_optimizer
    params, state, action, R, cfg = case(3, 8, wscale=2.0)
    eng = engine()
    eng.load_params(params)
    o = make_optimizer(opt, 1e-3, beta1=0.8, beta2=0.75, epsilon=1e-8)
    ref_p = {k: v.copy() for k, v in params.items()}
    ref_s = O.init_slots(ref_p, opt, beta1=0.8, beta2=0.75)
    upd_scale = {k: 0.0 for k in ref_p}
    for step in range(3):
        prev = {k: v.astype(np.float64) for k, v in ref_p.items()}
        eng.train_grads(dev(state), dev(action), dev(R))
        g = {k: O.clip_by_average_norm(v) for k, v in eng.state_dict(eng.grads).items()}
        o.apply_gradients(eng, fuse_clip=True)
        for k in ref_p:
            if opt == "adam":
                ref_p[k], ref_s["m"][k], ref_s["v"][k] = O.apply_adam(
                    ref_p[k], g[k], ref_s["m"][k], ref_s["v"][k], 1e-3, 0.8, 0.75, 1e-8,
                    ref_s["beta1_power"], ref_s["beta2_power"])
            elif opt == "rms":
                ref_p[k], ref_s["ms"][k], ref_s["mom"][k] = O.apply_rmsprop(
                    ref_p[k], g[k], ref_s["ms"][k], ref_s["mom"][k], 1e-3)
            elif opt == "gd":
                ref_p[k] = O.apply_gd(ref_p[k], g[k], 1e-3)
            elif opt == "momentum":
                ref_p[k], ref_s["accum"][k] = O.apply_momentum(ref_p[k], g[k], ref_s["accum"][k], 1e-3)
            elif opt == "adagrad":
                ref_p[k], ref_s["accum"][k] = O.apply_adagrad(ref_p[k], g[k], ref_s["accum"][k], 1e-3)
            else:
                ref_p[k], ref_s["accum"][k], ref_s["accum_update"][k] = O.apply_adadelta(
                    ref_p[k], g[k], ref_s["accum"][k], ref_s["accum_update"][k], 1e-3, eps=1e-3)
        if opt == "adam":
            ref_s["beta1_power"] = np.float32(ref_s["beta1_power"] * np.float32(0.8))
            ref_s["beta2_power"] = np.float32(ref_s["beta2_power"] * np.float32(0.75))
        got = eng.state_dict()
        for k in ref_p:
            # both sides round p to fp32 after the same functor arithmetic: allow the update
            # tolerance (relative to the largest per-step update so far) plus a few ulps of p
            upd_scale[k] = max(upd_scale[k], float(np.abs(ref_p[k] - prev[k]).max()))
            err = np.abs(got[k].astype(np.float64) - ref_p[k])
            lim = GRAD_TOL * upd_scale[k] + 4 * np.spacing(np.abs(ref_p[k]).astype(np.float32))
            bad = err > lim
            assert not bad.any(), (opt, step, k, got[k][bad][:4], ref_p[k][bad][:4],
                                   params[k][bad][:4], g[k][bad][:4])


def test_end_to_end_adam_step_vs_oracle_train_step():
    """One full step (fwd+bwd+clip+Adam, README best hyper-parameters) against the oracle's
    train_step: gradients within 1e-4; parameter updates compared where the oracle gradient is
    not at the rounding floor (Adam maps |g| >> eps to ~sign(g), so a g ~ 1e-9 whose sign
    differs between two correct fp32 evaluations would flip its update)."""
    from ba3c_amd.optimizer import AdamOptimizer
    params, state, action, R, cfg = case(21, 32, wscale=2.0)
    eng = engine()
    eng.load_params(params)
    opt = AdamOptimizer(1e-3, beta1=0.8, beta2=0.75, epsilon=1e-8)
    eng.train_grads(dev(state), dev(action), dev(R))
    opt.apply_gradients(eng, fuse_clip=True)
    got = eng.state_dict()
    slots = O.init_slots(as64(params), "adam", 0.8, 0.75)
    newp, _, _, g = O.train_step(as64(params), slots, 1, [(state, action, R.astype(np.float64))], cfg,
                                 lr=1e-3, beta1=0.8, beta2=0.75, eps=1e-8)
    for k in g:
        d_got = got[k].astype(np.float64) - params[k]
        d_ref = newp[k] - params[k]
        mask = np.abs(g[k]) > 1e-4 * max(np.abs(g[k]).max(), 1e-30)
        if mask.any():
            assert rel(d_got[mask], d_ref[mask]) < GRAD_TOL, k


@pytest.mark.parametrize("A", [2, 4, 18])
def test_sampling_bit_exact_vs_numpy_choice(A):
    eng = engine()
    rs = np.random.RandomState(A)
    probs = rs.dirichlet(np.ones(A) * 0.3, size=4096).astype(np.float32)
    probs[::13] = 0
    probs[::13, A - 1] = 1.0
    a_ref = O.np_random_choice(probs, np.random.RandomState(99))
    u = O.draw_uniforms(len(probs), np.random.RandomState(99))
    actions, flag = eng.sample(dev(probs), dev(u))
    assert int(flag.item()) == 0
    np.testing.assert_array_equal(actions.cpu().numpy(), a_ref)


def test_sampling_flags_nonfinite_and_bad_sum():
    eng = engine()
    probs = np.full((3, 4), 0.25, np.float32)
    probs[1, 2] = np.nan
    probs[2] = [0.5, 0.5, 0.5, 0.0]
    _, flag = eng.sample(dev(probs), dev(np.full(3, 0.3)))
    assert int(flag.item()) & 1 and int(flag.item()) & 2


def test_maxpool_ties_route_gradient_to_first_max():
    """Constant frames make every conv0 window tie: the gradient must go to the FIRST max of
    each window (TF's MaxPoolGrad), exactly as the oracle routes it."""
    params, _, action, R, cfg = case(5, 4, wscale=1.0)
    params["conv0/W"] = np.abs(params["conv0/W"])          # positive outputs everywhere
    state = np.full((4, 84, 84, 4), 200, np.uint8)
    state[1, :, ::2] = 17                                   # ties along rows only
    eng = engine()
    eng.load_params(params)
    eng.train_grads(dev(state), dev(action), dev(R))
    t, _, g = O.loss_and_grads(as64(params), state, action, R.astype(np.float64), cfg)
    got = eng.state_dict(eng.grads)
    _, codes = gpu_decisions(eng, 4)
    for layer in range(3):      # identical routing decisions on exact ties
        np.testing.assert_array_equal(codes[layer], np.where(t["p%d" % layer] > 0, t["c%d" % layer], 255))
    for k in g:
        assert rel(got[k], g[k]) < GRAD_TOL, k
