"""Oracle self-consistency: finite differences, an independent torch-autograd restatement,
TF-semantics spot checks and numpy's own RandomState.choice (the only pinned piece).

The reference ships no golden vectors for this path: the network,
loss, clip and optimizer restatement is "parity unpinned" by the reference itself.
"""
import numpy as np
import pytest
import torch

from oracle import ba3c_oracle as O

CFG = {"fc_neurons": 16, "fc_splits": 2, "replace_with_conv": True}


def _small_case(seed=0, B=3, C=4, A=4, dtype=np.float64, cfg=CFG, scale=3.0):
    rs = np.random.RandomState(seed)
    params = O.init_params(cfg["fc_neurons"], cfg.get("fc_splits", 1), A, seed=seed,
                           replace_with_conv=cfg.get("replace_with_conv", True),
                           ps=cfg.get("ps", 1), dtype=dtype)
    # larger weights so ReLUs/pools are non-trivial on random frames
    for k in params:
        params[k] = params[k] * dtype(scale)
    state = rs.randint(0, 256, size=(B, 84, 84, C)).astype(np.uint8)
    action = rs.randint(0, A, size=B).astype(np.int64)
    R = rs.normal(size=B).astype(dtype)
    return params, state, action, R


def _cost(params, state, action, R, cfg, adv=None):
    t, sc = O.build_graph_cost(params, state, action, R, cfg, frozen_advantage=adv)
    return sc["cost"]


@pytest.mark.parametrize("cfg", [CFG, {"fc_neurons": 12, "fc_splits": 1, "replace_with_conv": False, "ps": 3}])
def test_backward_matches_finite_differences(cfg):
    params, state, action, R = _small_case(cfg=cfg, scale=1.0)
    t, _, g = O.loss_and_grads(params, state, action, R, cfg)
    adv = t["adv"].copy()      # stop_gradient(V) - R is a constant for the derivative
    rs = np.random.RandomState(1)
    for name in params:
        p = params[name]
        flat = p.reshape(-1)
        idx = rs.choice(flat.size, size=min(6, flat.size), replace=False)
        if name == "conv0/W":   # include a padded channel (zero gradient) and a real one
            idx = np.concatenate([idx, [np.ravel_multi_index((2, 2, 0, 3), p.shape),
                                        np.ravel_multi_index((1, 3, 9, 5), p.shape)]])
        for i in idx:
            old = flat[i]
            h = 1e-6 * max(1.0, abs(old))
            flat[i] = old + h
            cp = _cost(params, state, action, R, cfg, adv)
            flat[i] = old - h
            cm = _cost(params, state, action, R, cfg, adv)
            flat[i] = old
            fd = (cp - cm) / (2 * h)
            flat[i] = old + h / 2
            cp2 = _cost(params, state, action, R, cfg, adv)
            flat[i] = old - h / 2
            cm2 = _cost(params, state, action, R, cfg, adv)
            flat[i] = old
            fd2 = (cp2 - cm2) / h
            if abs(fd - fd2) > 1e-6 * max(1.0, abs(fd)):
                continue            # a ReLU/max-pool kink inside the stencil: FD undefined
            an = g[name].reshape(-1)[i]
            assert abs(fd - an) <= 1e-5 * max(1.0, abs(an)) + 1e-8, (name, i, fd, an)


def _torch_cost(params_t, state, action, R, cfg):
    """Independent restatement with torch ops (NCHW convs) for the autograd cross-check."""
    x = torch.from_numpy(state.astype(np.float64)) / 255.0
    B, _, _, C = x.shape
    x = torch.cat([x, torch.zeros(B, 84, 84, 16 - C, dtype=x.dtype)], dim=3).permute(0, 3, 1, 2)

    def conv(z, w):
        return torch.nn.functional.conv2d(z, w.permute(3, 2, 0, 1))

    def pool(z):
        return torch.nn.functional.max_pool2d(z, 2)

    l = pool(torch.relu(conv(x, params_t["conv0/W"])))
    l = pool(torch.relu(conv(l, params_t["conv1/W"])))
    l = pool(torch.relu(conv(l, params_t["conv2/W"])))
    l = torch.relu(conv(l, params_t["conv3/W"]))
    S = cfg["fc_splits"]
    hs = [conv(l, params_t["fc1_%d/W" % i]).reshape(B, -1) for i in range(S)]
    h = torch.cat(hs, dim=1)
    pol = h @ params_t["fc-pi/W"] + params_t["fc-pi/b"]
    V = (h @ params_t["fc-v/W"] + params_t["fc-v/b"])[:, 0]
    p = torch.softmax(pol, dim=1)
    logp = torch.log(p + 1e-6)
    Rt = torch.from_numpy(R)
    lpa = (logp * torch.nn.functional.one_hot(torch.from_numpy(action), p.shape[1])).sum(1)
    adv = V.detach() - Rt
    cost = ((lpa * adv).sum() + 0.01 * (p * logp).sum() + 0.5 * ((V - Rt) ** 2).sum()) / B
    return cost, p, V


def test_oracle_matches_torch_autograd():
    params, state, action, R = _small_case(seed=3, B=4)
    t, sc, g = O.loss_and_grads(params, state, action, R, CFG)
    pt = {k: torch.tensor(v, requires_grad=True) for k, v in params.items()}
    cost, p, V = _torch_cost(pt, state, action, R, CFG)
    cost.backward()
    assert abs(cost.item() - sc["cost"]) < 1e-12 * max(1, abs(sc["cost"]))
    np.testing.assert_allclose(p.detach().numpy(), t["logits"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(V.detach().numpy(), t["pred_value"], rtol=1e-12, atol=1e-14)
    for k in params:
        ref = pt[k].grad.numpy()
        err = np.abs(ref - g[k]).max() / max(np.abs(ref).max(), 1e-30)
        assert err < 1e-10, (k, err)


def test_maxpool_first_max_tie_rule():
    x = np.zeros((1, 4, 4, 1))
    x[0, 0, 0, 0] = 2.0
    x[0, 0, 1, 0] = 2.0          # tie in window (0,0): first in row-major order wins
    x[0, 1, 0, 0] = 2.0
    x[0, 2, 3, 0] = 1.0          # window (1,1): max at sub (0,1)
    x[0, 3, 2, 0] = 1.0          # tie with (1,0): row-major first is (0,1)
    pooled, code = O.maxpool2x2_argmax(x)
    assert code[0, 0, 0, 0] == 0 and code[0, 1, 1, 0] == 1
    d = O.maxpool2x2_backward(np.ones_like(pooled), code, (4, 4))
    assert d[0, 0, 0, 0] == 1 and d[0, 0, 1, 0] == 0 and d[0, 1, 0, 0] == 0
    assert d[0, 2, 3, 0] == 1 and d[0, 3, 2, 0] == 0


def test_clip_by_average_norm_tf_formula():
    g = np.array([[3.0, 4.0]], dtype=np.float32)           # ||g|| = 5, n = 2
    out = O.clip_by_average_norm(g, 0.1)
    # (g*0.1)*min(2/5, 10) = g*0.04
    np.testing.assert_allclose(out, g * np.float32(0.1) * np.float32(0.4), rtol=1e-7)
    tiny = np.full((100,), 1e-4, dtype=np.float32)         # n/||g|| = 1e5 > 10 -> unchanged
    np.testing.assert_allclose(O.clip_by_average_norm(tiny), tiny, rtol=1e-6)
    zero = np.zeros((7,), dtype=np.float32)
    assert not np.isnan(O.clip_by_average_norm(zero)).any()


def test_adam_tf_form_differs_from_textbook_and_matches_closed_form():
    p = np.array([1.0, -2.0], np.float32)
    g = np.array([0.5, 0.25], np.float32)
    m = np.zeros_like(p)
    v = np.zeros_like(p)
    lr, b1, b2, eps = 1e-3, 0.8, 0.75, 1e-8
    p1, m1, v1 = O.apply_adam(p, g, m, v, lr, b1, b2, eps, np.float32(b1), np.float32(b2))
    alpha = np.float32(lr) * np.sqrt(np.float32(1 - b2)) / np.float32(1 - b1)
    exp = p - (np.float32(1 - b1) * g * alpha) / (np.sqrt(np.float32(1 - b2) * g * g) + np.float32(eps))
    np.testing.assert_allclose(p1, exp, rtol=1e-6)


def test_sample_from_u_matches_numpy_choice_bit_exact():
    rs = np.random.RandomState(0)
    probs = rs.dirichlet(np.ones(4), size=2000).astype(np.float32)
    probs[::7] = np.array([0.0, 1.0, 0.0, 0.0], np.float32)   # degenerate rows
    probs[::11] = np.float32(0.25)
    a_ref = O.np_random_choice(probs, np.random.RandomState(123))
    u = O.draw_uniforms(len(probs), np.random.RandomState(123))
    np.testing.assert_array_equal(O.sample_from_u(probs, u), a_ref)


def test_train_step_sync_mean_of_clipped():
    params, state, action, R = _small_case(seed=5, B=2, dtype=np.float32)
    slots = O.init_slots(params, "adam")
    b = [(state, action, R), (state[::-1].copy(), action[::-1].copy(), R[::-1].copy())]
    newp, news, sc, g = O.train_step(params, slots, 1, b, CFG)
    _, _, g0 = O.loss_and_grads(params, *b[0], CFG)
    _, _, g1 = O.loss_and_grads(params, *b[1], CFG)
    for k in params:
        exp = (O.clip_by_average_norm(g0[k]) + O.clip_by_average_norm(g1[k])) / np.float32(2)
        np.testing.assert_allclose(g[k], exp, rtol=1e-6, atol=1e-12)
    assert news["beta1_power"] == np.float32(np.float32(0.8) * np.float32(0.8))


def test_chunked_oracle_equals_whole_batch():
    """loss_and_grads_chunked (used to pin large-batch GPU steps) reproduces the whole-batch
    oracle: gradients and scalars combine by the batch-mean weights of train.py:299,326."""
    params, state, action, R = _small_case(seed=4, B=7, scale=2.0)
    _, sc, g = O.loss_and_grads(params, state, action, R, CFG)
    t2, sc2, g2 = O.loss_and_grads_chunked(params, state, action, R, CFG, chunk=3)
    for k in g:
        np.testing.assert_allclose(g2[k], g[k], rtol=1e-11, atol=1e-15)
    for k in sc:
        assert abs(float(sc2[k]) - float(sc[k])) <= 1e-11 * max(1.0, abs(float(sc[k]))), k
    assert t2["logits"].shape == (7, 4) and t2["own_c0"].shape == (7, 40, 40, 32)


def test_torch_cpu_baseline_restatement_matches_oracle():
    """oracle/ba3c_torch_cpu.py (the timed CPU baseline) computes the same step as the numpy
    oracle: raw gradients within 1e-4 and one clip+Adam update within 1e-4 of the update."""
    from oracle.ba3c_torch_cpu import TorchCpuBa3c
    cfg = {"fc_neurons": 16, "fc_splits": 2}
    p32 = O.init_params(16, 2, 4, seed=2, dtype=np.float32)
    for k in p32:
        p32[k] = p32[k] * np.float32(2.0)
    rs = np.random.RandomState(5)
    state = rs.randint(0, 256, size=(3, 84, 84, 4)).astype(np.uint8)
    action = rs.randint(0, 4, size=3).astype(np.int64)
    R = rs.normal(size=3).astype(np.float32)
    m = TorchCpuBa3c(p32, 16, 2)
    st, ac, rr = torch.from_numpy(state), torch.from_numpy(action), torch.from_numpy(R)
    cost, g = m.loss_and_grads(st, ac, rr)
    p64 = {k: v.astype(np.float64) for k, v in p32.items()}
    _, sc, gref = O.loss_and_grads(p64, state, action, R.astype(np.float64), cfg)
    assert abs(float(cost) - sc["cost"]) < 1e-5 * max(1.0, abs(sc["cost"]))
    for k in gref:
        err = np.abs(g[k].numpy() - gref[k]).max() / max(np.abs(gref[k]).max(), 1e-30)
        assert err < 1e-4, (k, err)
    m.step(st, ac, rr)
    newp, _, _, gc = O.train_step(p64, O.init_slots(p64, "adam", 0.8, 0.75), 1,
                                  [(state, action, R.astype(np.float64))], cfg)
    for k in newp:
        d_got = m.p[k].numpy().astype(np.float64) - p32[k]
        d_ref = newp[k] - p64[k]
        mask = np.abs(gc[k]) > 1e-4 * max(np.abs(gc[k]).max(), 1e-30)
        if mask.any():
            e = np.abs(d_got[mask] - d_ref[mask]).max() / np.abs(d_ref[mask]).max()
            assert e < 1e-4, (k, e)


@pytest.mark.parametrize("frames", ["random", "atari"])
def test_torch_f64_forced_restatement_matches_oracle(frames):
    """oracle/ba3c_torch_f64.py (the checker of the B=2048 GPU test) against the numpy oracle:
    the same forced decisions (the oracle's own, so both follow one routing), every gradient
    and the cost to ~1e-12; its own_decisions() equal the oracle's own codes and ReLU signs."""
    from atari_frames import atari_frames
    from oracle.ba3c_torch_f64 import loss_and_grads_forced, own_decisions
    B = 6
    rs = np.random.RandomState(9)
    p32 = O.init_params(512, 1, 4, seed=2, dtype=np.float32)
    params = {k: v.astype(np.float64) for k, v in p32.items()}
    state = (atari_frames(B, 3) if frames == "atari"
             else rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8))
    action = rs.randint(0, 4, size=B)
    R = rs.normal(size=B)
    cfg = {"fc_neurons": 512, "fc_splits": 1}
    t, s, g = O.loss_and_grads_chunked(params, state, action, R, cfg, chunk=4)
    forced = {"c0": t["own_c0"], "c1": t["own_c1"], "c2": t["own_c2"], "a3_mask": t["a3_pos"]}
    g2, out = loss_and_grads_forced(params, state, action, R, cfg, forced, chunk=4)
    for k in g:
        assert np.abs(g[k] - g2[k]).max() <= 1e-11 * np.abs(g[k]).max(), k
    assert abs(out["cost"] - s["cost"]) <= 1e-12 * max(1.0, abs(s["cost"]))
    own = own_decisions(p32, state, chunk=4)
    for k in ("c0", "c1", "c2", "a3_mask"):
        np.testing.assert_array_equal(own[k], forced[k])
    for k in ("near_c0", "near_c1", "near_c2", "near_a3"):
        np.testing.assert_array_equal(own[k], t[k])
