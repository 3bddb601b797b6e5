"""CPU oracle for the BA3C learner/predictor hot path — TEST INFRASTRUCTURE ONLY.

This module is a numpy restatement of the reference TensorFlow-1.2 graph built by
`/root/reference/src/OpenAIGym/train.py` (Model, lines 144-330) plus the optimizer
(`train.py:582-606`) and the action sampler (`train.py:374-392`).  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it, and only
as the checker / CPU baseline — never as the product path.

PARITY STATUS: **parity unpinned** for the network, loss, clip and optimizer.  The
reference ships no tests, golden vectors or fixtures for this path, TensorFlow 1.2.1 is
not installed in this image and the reference sources are Python-2 only.
The restatement is written from the reference graph plus TF-1.2 op semantics
 and is cross-checked in `tests/` against (a) central finite
differences in float64 and (b) an independent torch-autograd restatement.
The action sampler IS pinned: `np_random_choice` calls numpy's own legacy
`RandomState.choice` (the exact library call of `train.py:382`), and `sample_from_u`
is checked against it draw for draw.

Arithmetic runs in the dtype of the parameters (float64 for golden vectors, float32 for
the CPU baseline).  Layout is TF's: NHWC activations, HWIO conv weights, [in,out] FC.
"""
import math

import numpy as np

# --- constants of the reference graph -------------------------------------------------
IMAGE_SIZE = (84, 84)           # train.py:92
FRAME_HISTORY = 4               # train.py:93
TARGET_CHANNELS = 16            # train.py:99 (input zero-padded to 16 channels)
LOG_EPS = 1e-6                  # train.py:305  log(p + 1e-6)
CLIP_NORM = 0.1                 # train.py:330  clip_by_average_norm(grad, 0.1)
MONITOR_SCALE = 128.0           # train.py:310,315,320  "* 128 / batch_size"


# --- parameter inventory (train.py:177-264) ---------------------------------------------
def param_specs(fc_neurons=512, fc_splits=1, num_actions=4, replace_with_conv=True, ps=1):
    """Ordered (name, shape) list of trainable variables, names = checkpoint keys.

    conv0..conv3: `train.py:177-212` (Conv2D, use_bias=False, HWIO).
    fc1_i:        `train.py:216-229` (S convs 5x5 on the 5x5x64 map, no bias) or the legacy
                  FullyConnected split of `train.py:230-243` (bias, ReLU, split by --ps).
    fc-pi, fc-v:  `train.py:250-264` (FullyConnected with bias, identity).
    """
    specs = [("conv0/W", (5, 5, TARGET_CHANNELS, 32)),
             ("conv1/W", (5, 5, 32, 32)),
             ("conv2/W", (5, 5, 32, 64)),
             ("conv3/W", (3, 3, 64, 64))]
    if replace_with_conv:
        assert fc_neurons % fc_splits == 0
        per = fc_neurons // fc_splits
        for i in range(fc_splits):
            specs.append(("fc1_%d/W" % i, (5, 5, 64, per)))
    else:
        assert fc_neurons % ps == 0
        per = fc_neurons // ps
        for i in range(ps):
            specs.append(("fc1_%d/W" % i, (1600, per)))
            specs.append(("fc1_%d/b" % i, (per,)))
    specs += [("fc-pi/W", (fc_neurons, num_actions)), ("fc-pi/b", (num_actions,)),
              ("fc-v/W", (fc_neurons, 1)), ("fc-v/b", (1,))]
    return specs


def _trunc_normal(rs, shape, std):
    out = rs.normal(0.0, std, size=shape)
    bad = np.abs(out) > 2 * std
    while bad.any():
        out[bad] = rs.normal(0.0, std, size=int(bad.sum()))
        bad = np.abs(out) > 2 * std
    return out


def init_params(fc_neurons=512, fc_splits=1, num_actions=4, seed=0, conv_init="normal",
                fc_init="uniform", replace_with_conv=True, ps=1, dtype=np.float32):
    """Reference initialisers (`models/conv2d.py:48-55`, `models/fc.py:35-38`), numpy RNG.

    TF's own random streams cannot be reproduced; parity always runs on identical weights
    handed to both sides, so only the distributions matter here.
    """
    rs = np.random.RandomState(seed)
    params = {}
    for name, shape in param_specs(fc_neurons, fc_splits, num_actions, replace_with_conv, ps):
        if name.endswith("/b"):
            v = np.zeros(shape)
        elif name.startswith("conv"):
            if conv_init == "normal":
                v = _trunc_normal(rs, shape, 3e-2)
            elif conv_init == "uniform":
                v = rs.uniform(-0.05, 0.05, size=shape)
            else:  # xavier_initializer_conv2d: fan_in = kh*kw*cin, fan_out = kh*kw*cout
                fan_in = shape[0] * shape[1] * shape[2]
                fan_out = shape[0] * shape[1] * shape[3]
                lim = math.sqrt(6.0 / (fan_in + fan_out))
                v = rs.uniform(-lim, lim, size=shape)
        elif name.startswith("fc1_") and replace_with_conv:
            # uniform_unit_scaling_initializer(1.43): U(+-1.43*sqrt(3/fan_in)), fan_in=1600
            lim = 1.43 * math.sqrt(3.0 / 1600.0)
            v = rs.uniform(-lim, lim, size=shape)
        else:
            fan_in = shape[0]
            if fc_init == "normal":
                v = _trunc_normal(rs, shape, 1.0 / math.sqrt(fan_in))
            else:
                lim = 1.43 * math.sqrt(3.0 / fan_in)
                v = rs.uniform(-lim, lim, size=shape)
        params[name] = np.asarray(v, dtype=dtype)
    return params


# --- layers -----------------------------------------------------------------------------
def _im2col(x, kh, kw):
    """x [B,H,W,C] -> [B,Ho,Wo,kh,kw,C] (VALID, stride 1) as a strided view."""
    B, H, W, C = x.shape
    Ho, Wo = H - kh + 1, W - kw + 1
    s = x.strides
    return np.lib.stride_tricks.as_strided(
        x, shape=(B, Ho, Wo, kh, kw, C), strides=(s[0], s[1], s[2], s[1], s[2], s[3]),
        writeable=False)


def conv2d_valid(x, w):
    """tf.nn.conv2d(x, W, [1,1,1,1], 'VALID') — `models/conv2d.py:63-66`, Appendix A.1."""
    kh, kw, ci, co = w.shape
    cols = _im2col(np.ascontiguousarray(x), kh, kw)
    B, Ho, Wo = cols.shape[:3]
    out = cols.reshape(B * Ho * Wo, kh * kw * ci) @ w.reshape(kh * kw * ci, co)
    return out.reshape(B, Ho, Wo, co)


def conv2d_valid_dgrad(dy, w, in_hw):
    """Conv2DBackpropInput: full correlation of dy with the spatially flipped kernel."""
    kh, kw, ci, co = w.shape
    B, Ho, Wo, _ = dy.shape
    pad = np.zeros((B, Ho + 2 * (kh - 1), Wo + 2 * (kw - 1), co), dtype=dy.dtype)
    pad[:, kh - 1:kh - 1 + Ho, kw - 1:kw - 1 + Wo, :] = dy
    wf = w[::-1, ::-1].transpose(0, 1, 3, 2)          # [kh,kw,co,ci]
    dx = conv2d_valid(pad, np.ascontiguousarray(wf))
    assert dx.shape[1:3] == tuple(in_hw)
    return dx


def conv2d_valid_wgrad(x, dy, kshape):
    """Conv2DBackpropFilter: dW[kh,kw,ci,co] = sum_{n,y,x} x[n,y+kh,x+kw,ci] dy[n,y,x,co]."""
    kh, kw = kshape
    cols = _im2col(np.ascontiguousarray(x), kh, kw)
    B, Ho, Wo = cols.shape[:3]
    ci = x.shape[3]
    co = dy.shape[3]
    dw = cols.reshape(B * Ho * Wo, kh * kw * ci).T @ dy.reshape(B * Ho * Wo, co)
    return dw.reshape(kh, kw, ci, co)


def maxpool2x2_argmax(x):
    """MaxPooling(x, 2) (`models/pool.py:14-33`): 2x2/2 VALID.

    Returns (pooled, code) where code in {0,1,2,3} is the row-major position of the first
    maximum of each window (TF CPU's strict-'<' update order, Appendix A.3).
    """
    B, H, W, C = x.shape
    win = x.reshape(B, H // 2, 2, W // 2, 2, C).transpose(0, 1, 3, 2, 4, 5)
    win = win.reshape(B, H // 2, W // 2, 4, C)
    code = np.argmax(win, axis=3)          # numpy argmax returns the FIRST maximum
    pooled = np.take_along_axis(win, code[:, :, :, None, :], axis=3)[:, :, :, 0, :]
    return pooled, code.astype(np.uint8)


def maxpool2x2_backward(dpooled, code, hw):
    """MaxPoolGrad: route each window's gradient to its recorded argmax position."""
    B, Hp, Wp, C = dpooled.shape
    win = np.zeros((B, Hp, Wp, 4, C), dtype=dpooled.dtype)
    np.put_along_axis(win, code[:, :, :, None, :].astype(np.int64),
                      dpooled[:, :, :, None, :], axis=3)
    win = win.reshape(B, Hp, Wp, 2, 2, C).transpose(0, 1, 3, 2, 4, 5)
    return win.reshape(B, hw[0], hw[1], C)


def relu(x):
    return np.maximum(x, 0)


def softmax(z):
    """tf.nn.softmax (Appendix A.5)."""
    z = z - z.max(axis=1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(axis=1, keepdims=True)


# --- network (train.py:164-272) ---------------------------------------------------------
def fc1_weight_matrix(params, fc_neurons, fc_splits):
    """concat_i reshape(W_i [5,5,64,F/S] -> [1600,F/S]) along axis 1 (`train.py:216-229`)."""
    mats = [params["fc1_%d/W" % i].reshape(1600, fc_neurons // fc_splits) for i in range(fc_splits)]
    return np.concatenate(mats, axis=1)


def get_nn_prediction(params, state, cfg, explore_factor=1.0):
    """Model._get_NN_prediction_wrapped (`train.py:164-272`) + softmax heads (`:286-295`).

    state: uint8 or float [B,84,84,C]; returns a dict of every intermediate the backward
    pass needs plus the predictor outputs 'logits' (softmax probs), 'logitsT', 'pred_value'.
    """
    dt = params["conv0/W"].dtype
    B = state.shape[0]
    C = state.shape[3]
    x = state.astype(dt) / dt.type(255.0)                                     # train.py:167
    x = np.concatenate([x, np.zeros((B, 84, 84, TARGET_CHANNELS - C), dt)], axis=3)  # :173-174
    t = {"x": x}
    z0 = conv2d_valid(x, params["conv0/W"])                                 # :177-178
    a0 = relu(z0)                                                           # :175
    p0, c0 = maxpool2x2_argmax(a0)                                          # :185
    z1 = conv2d_valid(p0, params["conv1/W"])                                # :187-188
    a1 = relu(z1)
    p1, c1 = maxpool2x2_argmax(a1)                                          # :195
    z2 = conv2d_valid(p1, params["conv2/W"])                                # :197-198
    a2 = relu(z2)
    p2, c2 = maxpool2x2_argmax(a2)                                          # :204
    z3 = conv2d_valid(p2, params["conv3/W"])                                # :206-207
    a3 = relu(z3)
    t.update(a0=a0, p0=p0, c0=c0, a1=a1, p1=p1, c1=c1, a2=a2, p2=p2, c2=c2, a3=a3,
             z0=z0, z1=z1, z2=z2, z3=z3)
    flat = a3.reshape(B, 1600)                                              # batch_flatten
    F = cfg["fc_neurons"]
    if cfg.get("replace_with_conv", True):
        W1 = fc1_weight_matrix(params, F, cfg["fc_splits"])
        h = flat @ W1                                                       # :216-229 identity
        t["h_pre"] = h
    else:
        nps = cfg.get("ps", 1)
        parts = []
        for i in range(nps):
            parts.append(flat @ params["fc1_%d/W" % i] + params["fc1_%d/b" % i])
        h_pre = np.concatenate(parts, axis=1)
        t["h_pre"] = h_pre
        h = relu(h_pre)                                                     # :238 relu1
    t["flat"] = flat
    t["h"] = h
    policy = h @ params["fc-pi/W"] + params["fc-pi/b"]                       # :250-252
    value = (h @ params["fc-v/W"] + params["fc-v/b"])[:, 0]                  # :257-259, :287
    t["policy"] = policy
    t["pred_value"] = value
    t["logits"] = softmax(policy)                                           # :288 (probs!)
    t["logitsT"] = softmax(policy * dt.type(explore_factor))                # :299
    relus = [a0, a1, a2, a3] + ([] if cfg.get("replace_with_conv", True) else [h])
    t["active_relus"] = int(sum(int(np.count_nonzero(r)) for r in relus))  # :271
    return t


# --- loss (train.py:274-327) ------------------------------------------------------------
def build_graph_cost(params, state, action, futurereward, cfg, entropy_beta=0.01,
                     frozen_advantage=None, forced_h=None):
    """Model._build_graph (`train.py:274-327`): returns (t, scalars) with t['cost'].

    `frozen_advantage` replaces stop_gradient(V) - R by a constant array, so a finite
    difference of `cost` sees exactly the function TF differentiates (`train.py:309`).
    `forced_h` (tests only, replace_with_conv FC) evaluates the heads, softmax and loss on a
    given FC output [B, F] — the checked side's own — so that the head / loss gradient is
    compared on its arithmetic alone where the policy saturates: there d(dz)/dz is
    exp-amplified and any fp32 forward (TF's included) moves dz by |dz| * |dlogit|.
    """
    t = get_nn_prediction(params, state, cfg)
    dt = params["conv0/W"].dtype
    if forced_h is not None:
        # the heads and the loss evaluated on the checked side's own FC output (tests only)
        h = forced_h.astype(dt)
        t["h"] = h
        t["policy"] = h @ params["fc-pi/W"] + params["fc-pi/b"]
        t["pred_value"] = (h @ params["fc-v/W"] + params["fc-v/b"])[:, 0]
        t["logits"] = softmax(t["policy"])
    p = t["logits"]
    V = t["pred_value"]
    R = futurereward.astype(dt)
    B = dt.type(p.shape[0])                                                  # :299
    A = p.shape[1]
    logp = np.log(p + dt.type(LOG_EPS))                                      # :305
    onehot = np.eye(A, dtype=dt)[action]
    lpa = (logp * onehot).sum(axis=1)                                        # :307-308
    adv = V - R if frozen_advantage is None else frozen_advantage           # :309 stop_grad(V)-R
    policy_loss = (lpa * adv).sum()                                          # :310
    xent = (p * logp).sum()                                                  # :314
    value_loss = ((V - R) ** 2).sum() / dt.type(2)                           # :319 l2_loss
    beta = dt.type(entropy_beta)
    cost = (policy_loss + xent * beta + value_loss) / B                      # :326-327
    t.update(logp=logp, adv=adv, onehot=onehot)
    scalars = {
        "cost": cost,
        "policy_loss": policy_loss * dt.type(MONITOR_SCALE) / B,             # :311
        "xentropy_loss": xent * dt.type(MONITOR_SCALE) / B * beta,           # :315-316
        "value_loss": value_loss * dt.type(MONITOR_SCALE) / B,               # :320
        "advantage": adv.mean(),                                             # :323
        "pred_reward": V.mean(),                                             # :321
        "max_logit": p.max(),                                                # :291
        "mean_value": V.mean(),                                              # :290
        "active_relus": t["active_relus"],                                  # :271
    }
    return t, scalars


def backward(params, t, cfg, entropy_beta=0.01):
    """TF autodiff of `cost` (`train/multigpu.py:85-86`) restated by hand (Appendix A.2-A.6).

    Returns {var_name: grad} for every trainable variable of `param_specs`.
    """
    dt = params["conv0/W"].dtype
    p, V, logp, adv, onehot = t["logits"], t["pred_value"], t["logp"], t["adv"], t["onehot"]
    B = dt.type(p.shape[0])
    beta = dt.type(entropy_beta)
    # d cost / d p  (A.6)
    gp = (adv[:, None] * onehot / (p + dt.type(LOG_EPS))
          + beta * (logp + p / (p + dt.type(LOG_EPS)))) / B
    dz = p * (gp - (gp * p).sum(axis=1, keepdims=True))                   # SoftmaxGrad
    dV = (V - t["R"]) / B if "R" in t else None
    return _backward_from_heads(params, t, cfg, dz, dV)


def _backward_from_heads(params, t, cfg, dz, dV):
    dt = params["conv0/W"].dtype
    g = {}
    h = t["h"]
    g["fc-pi/W"] = h.T @ dz
    g["fc-pi/b"] = dz.sum(axis=0)
    g["fc-v/W"] = h.T @ dV[:, None]
    g["fc-v/b"] = np.array([dV.sum()], dtype=dt)
    dh = dz @ params["fc-pi/W"].T + dV[:, None] @ params["fc-v/W"].T
    F, S = cfg["fc_neurons"], cfg.get("fc_splits", 1)
    flat = t["flat"]
    if cfg.get("replace_with_conv", True):
        W1 = fc1_weight_matrix(params, F, S)
        dW1 = flat.T @ dh
        per = F // S
        for i in range(S):
            g["fc1_%d/W" % i] = dW1[:, i * per:(i + 1) * per].reshape(5, 5, 64, per)
        dflat = dh @ W1.T
    else:
        dh = dh * (t["h_pre"] > 0)
        nps = cfg.get("ps", 1)
        per = F // nps
        dflat = np.zeros_like(flat)
        for i in range(nps):
            sl = dh[:, i * per:(i + 1) * per]
            g["fc1_%d/W" % i] = flat.T @ sl
            g["fc1_%d/b" % i] = sl.sum(axis=0)
            dflat += sl @ params["fc1_%d/W" % i].T
    Bn = flat.shape[0]
    forced = t.get("forced")

    def pool_back(dp, layer, hw, act):
        if forced is None:
            return maxpool2x2_backward(dp, t["c%d" % layer], hw) * (act > 0)
        # the checked side's own discrete decisions: code 255 = window max <= 0 (no gradient)
        c = forced["c%d" % layer]
        return maxpool2x2_backward(np.where(c == 255, 0, dp), np.where(c == 255, 0, c), hw)

    mask3 = (t["a3"] > 0) if forced is None else forced["a3_mask"]
    da3 = dflat.reshape(Bn, 5, 5, 64) * mask3                               # ReluGrad (A.2)
    g["conv3/W"] = conv2d_valid_wgrad(t["p2"], da3, (3, 3))
    dp2 = conv2d_valid_dgrad(da3, params["conv3/W"], (7, 7))
    da2 = pool_back(dp2, 2, (14, 14), t["a2"])
    g["conv2/W"] = conv2d_valid_wgrad(t["p1"], da2, (5, 5))
    dp1 = conv2d_valid_dgrad(da2, params["conv2/W"], (18, 18))
    da1 = pool_back(dp1, 1, (36, 36), t["a1"])
    g["conv1/W"] = conv2d_valid_wgrad(t["p0"], da1, (5, 5))
    dp0 = conv2d_valid_dgrad(da1, params["conv1/W"], (40, 40))
    da0 = pool_back(dp0, 0, (80, 80), t["a0"])
    g["conv0/W"] = conv2d_valid_wgrad(t["x"], da0, (5, 5))                  # incl. padded ch.
    t.update(dz=dz, dV=dV, dh=dh, da3=da3, dp2=dp2, dp1=dp1, dp0=dp0)
    return g


def loss_and_grads(params, state, action, futurereward, cfg, entropy_beta=0.01, forced=None):
    """One tower's forward + loss + raw gradients (before the gradient processor).

    `forced` (tests only) = {'c0','c1','c2': uint8 argmax codes with 255 for max<=0,
    'a3_mask': bool} replaces the oracle's own max-pool / ReLU decisions in the backward pass,
    so an fp32 implementation can be compared on arithmetic alone when a near-tie or a
    pre-activation within rounding of zero resolves differently in fp32 and fp64."""
    fh = None if forced is None else forced.get("h")
    assert fh is None or cfg.get("replace_with_conv", True), "forced h: identity FC only"
    t, scalars = build_graph_cost(params, state, action, futurereward, cfg, entropy_beta,
                                  forced_h=fh)
    t["R"] = futurereward.astype(params["conv0/W"].dtype)
    if forced is not None:
        t["forced"] = forced
    grads = backward(params, t, cfg, entropy_beta)
    return t, scalars, grads


def loss_and_grads_chunked(params, state, action, futurereward, cfg, entropy_beta=0.01,
                           forced=None, chunk=16):
    """loss_and_grads over a large batch evaluated in sub-batches of <= `chunk` samples (memory
    stays at one chunk's im2col).  The cost is a mean over the batch (train.py:299,326-327), so
    the full-batch gradient is sum_c (B_c/B) grad_c, and the scalars combine the same way
    (means weighted, max_logit maxed, active_relus summed).  Returns (t, scalars, grads) with t
    holding the per-sample outputs ('logits', 'pred_value') and the oracle's own discrete
    decisions ('own_c0'..'own_c2': argmax codes with 255 where the window max <= 0, 'a3_pos')
    and where those decisions are numerically ambiguous ('near_c0'..'near_c2', 'near_a3', see
    ambiguous_windows)."""
    B = state.shape[0]
    dt = params["conv0/W"].dtype
    grads, sc = None, None
    keep = {"logits": [], "pred_value": [], "own_c0": [], "own_c1": [], "own_c2": [], "a3_pos": [],
            "near_c0": [], "near_c1": [], "near_c2": [], "near_a3": []}
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        f = None if forced is None else {k: v[lo:hi] for k, v in forced.items()}
        t, s, g = loss_and_grads(params, state[lo:hi], action[lo:hi], futurereward[lo:hi], cfg,
                                 entropy_beta, forced=f)
        w = dt.type(hi - lo) / dt.type(B)
        if grads is None:
            grads = {k: v * w for k, v in g.items()}
            sc = {k: (v if k in ("max_logit", "active_relus") else v * w) for k, v in s.items()}
        else:
            for k in g:
                grads[k] = grads[k] + g[k] * w
            for k, v in s.items():
                if k == "max_logit":
                    sc[k] = max(sc[k], v)
                elif k == "active_relus":
                    sc[k] += v
                else:
                    sc[k] = sc[k] + v * w
        keep["logits"].append(t["logits"])
        keep["pred_value"].append(t["pred_value"])
        for layer in range(3):
            keep["own_c%d" % layer].append(np.where(t["p%d" % layer] > 0, t["c%d" % layer], 255))
            keep["near_c%d" % layer].append(ambiguous_windows(t["z%d" % layer]))
        keep["a3_pos"].append(t["a3"] > 0)
        keep["near_a3"].append(ambiguous_relu(t["z3"]))
    return {k: np.concatenate(v) for k, v in keep.items()}, sc, grads


def _image_scale(z):
    return np.abs(z).reshape(z.shape[0], -1).max(axis=1).reshape((-1,) + (1,) * (z.ndim - 1))


def ambiguous_windows(z, tol=2e-5):
    """Max-pool windows of the pre-ReLU conv output z [B,H,W,C] whose first-max / ReLU
    decision an fp32 evaluation may legitimately resolve differently from this fp64 one: a
    window max within tol * (the image's max |z|) of zero (but not exactly zero: an all-zero
    patch is zero in any arithmetic), or a competitor that is NOT exactly
    equal to the max but within that distance of it (a near-tie).  Exact ties are not
    ambiguous: identical patches give identical values in any arithmetic.  Returns a bool mask
    of the pooled shape [B,H/2,W/2,C]."""
    B, H, W, C = z.shape
    win = z.reshape(B, H // 2, 2, W // 2, 2, C).transpose(0, 1, 3, 5, 2, 4).reshape(B, H // 2, W // 2, C, 4)
    eps = tol * _image_scale(z)[..., None]
    m = win.max(axis=-1, keepdims=True)
    gap = m - win
    near_tie = ((gap > 0) & (gap <= eps)).any(axis=-1)
    near_zero = (m[..., 0] != 0) & (np.abs(m[..., 0]) <= eps[..., 0])   # exact zeros: zero patches
    return near_tie | near_zero


def ambiguous_relu(z, tol=2e-5):
    """Pre-activations within tol * (the image's max |z|) of zero (ReLU sign decision)."""
    return (z != 0) & (np.abs(z) <= tol * _image_scale(z))


# --- gradient processor (train.py:329-330, tfutils/gradproc.py:34-67) --------------------
def clip_by_average_norm(g, clip_norm=CLIP_NORM):
    """tf.clip_by_average_norm (Appendix A.9): (t*c) * min(rsqrt(sum t^2) * n, 1/c)."""
    dt = g.dtype
    n = dt.type(g.size)
    ss = (g.astype(np.float64) ** 2).sum()
    inv = dt.type(np.inf) if ss == 0 else dt.type(1.0 / math.sqrt(ss))
    m = min(inv * n, dt.type(1.0) / dt.type(clip_norm))
    return (g * dt.type(clip_norm)) * dt.type(m)


# --- optimizers (train.py:582-597; TF-1.2 ApplyAdam / ApplyRMSProp CPU functors) ---------
def adam_alpha(lr, beta1_power, beta2_power):
    """alpha = lr*sqrt(1-b2p)/(1-b1p), evaluated in float32 as TF does (Appendix A.7)."""
    f = np.float32
    return f(f(lr) * np.sqrt(f(1) - f(beta2_power))) / (f(1) - f(beta1_power))


def apply_adam(p, g, m, v, lr, beta1, beta2, eps, beta1_power, beta2_power):
    """One ApplyAdam (Appendix A.7). beta*_power are the values BEFORE this step (b^t)."""
    dt = p.dtype
    alpha = dt.type(adam_alpha(lr, beta1_power, beta2_power))
    m = m + (g - m) * dt.type(1 - np.float32(beta1))
    v = v + (g * g - v) * dt.type(1 - np.float32(beta2))
    p = p - (m * alpha) / (np.sqrt(v) + dt.type(eps))
    return p, m, v


def apply_rmsprop(p, g, ms, mom, lr, decay=0.9, momentum=0.0, eps=1e-10):
    """ApplyRMSProp (Appendix A.8); `ms` slot is initialised to ones by the caller."""
    dt = p.dtype
    ms = ms + (g * g - ms) * dt.type(1 - np.float32(decay))
    mom = mom * dt.type(momentum) + (g * dt.type(lr)) / np.sqrt(ms + dt.type(eps))
    return p - mom, ms, mom


def apply_gd(p, g, lr):
    return p - g * p.dtype.type(lr)


def apply_momentum(p, g, accum, lr, momentum=0.9):
    """ApplyMomentum (use_nesterov=False): accum = accum*mu + g; var -= lr*accum."""
    accum = accum * p.dtype.type(momentum) + g
    return p - accum * p.dtype.type(lr), accum


def apply_adagrad(p, g, accum, lr):
    """ApplyAdagrad: accum += g^2; var -= lr*g*rsqrt(accum) (accum initialised to 0.1)."""
    accum = accum + g * g
    return p - g * p.dtype.type(lr) / np.sqrt(accum), accum


def apply_adadelta(p, g, accum, accum_update, lr, rho=0.95, eps=1e-3):
    """ApplyAdadelta (TF-1.2 CPU functor); slots initialised to 0."""
    dt = p.dtype
    accum = accum * dt.type(rho) + g * g * dt.type(1 - rho)
    update = np.sqrt(accum_update + dt.type(eps)) / np.sqrt(accum + dt.type(eps)) * g
    accum_update = accum_update * dt.type(rho) + update * update * dt.type(1 - rho)
    return p - update * dt.type(lr), accum, accum_update


# --- synchronous aggregation (train.py:598-606; train/multigpu.py:41-53) -----------------
def sync_replicas_mean(clipped_grads_per_replica):
    """SyncReplicasOptimizer with num_grad == n_workers: mean of already-clipped grads."""
    n = len(clipped_grads_per_replica)
    out = {}
    for k in clipped_grads_per_replica[0]:
        s = sum(r[k] for r in clipped_grads_per_replica)
        out[k] = s / s.dtype.type(n)
    return out


# --- action sampling (train.py:382) -------------------------------------------------------
def np_random_choice(probs, rs):
    """The reference's exact call: np.random.choice(len(p), p=p), once per state."""
    return np.array([rs.choice(len(pi), p=pi) for pi in probs], dtype=np.int64)


def draw_uniforms(n, rs):
    """The one MT19937 double `choice` consumes per call (legacy RandomState stream)."""
    return np.array([rs.random_sample() for _ in range(n)], dtype=np.float64)


def sample_from_u(probs, u):
    """numpy legacy `choice(p=...)` given its uniform draw u: searchsorted(cdf/cdf[-1], u, 'right')."""
    out = np.empty(probs.shape[0], dtype=np.int64)
    for i in range(probs.shape[0]):
        cdf = np.cumsum(probs[i].astype(np.float64))
        cdf /= cdf[-1]
        out[i] = np.searchsorted(cdf, u[i], side="right")
    return out


# --- full train step (trainer.py:244-299 -> one sess.run of TfDictOp) ---------------------
def train_step(params, slots, step_t, batches, cfg, opt="adam", lr=1e-3, beta1=0.8,
               beta2=0.75, eps=1e-8, entropy_beta=0.01, aggregate=None):
    """forward+backward per replica -> per-replica clip -> mean -> one optimizer apply.

    `batches` is a list of (state, action, R) per replica (1 entry = single worker).
    `aggregate`: indices of the replicas whose clipped grads enter the mean (backup workers,
    SyncReplicasOptimizer replicas_to_aggregate < total_num_replicas, train.py:601-602: the
    accumulator of TF 1.2's sync_replicas_optimizer.py — not vendored in the reference —
    averages the first replicas_to_aggregate fresh gradients and drops the stale rest);
    None = all replicas.
    `slots` holds optimizer state; beta powers follow TF's float32 variables.
    Returns (new_params, new_slots, scalars of replica 0, clipped-mean grads).
    """
    per = []
    sc0 = None
    for (state, action, R) in batches:
        _, sc, g = loss_and_grads(params, state, action, R, cfg, entropy_beta)
        per.append({k: clip_by_average_norm(v) for k, v in g.items()})
        if sc0 is None:
            sc0 = sc
    if aggregate is not None:
        per = [per[i] for i in aggregate]
    g = per[0] if len(per) == 1 else sync_replicas_mean(per)
    newp, news = {}, {k: dict(v) if isinstance(v, dict) else v for k, v in slots.items()}
    f32 = np.float32
    if opt == "adam":
        b1p, b2p = slots["beta1_power"], slots["beta2_power"]
        for k in params:
            newp[k], news["m"][k], news["v"][k] = apply_adam(
                params[k], g[k], slots["m"][k], slots["v"][k], lr, beta1, beta2, eps, b1p, b2p)
        news["beta1_power"] = f32(f32(b1p) * f32(beta1))
        news["beta2_power"] = f32(f32(b2p) * f32(beta2))
    elif opt == "rms":
        for k in params:
            newp[k], news["ms"][k], news["mom"][k] = apply_rmsprop(
                params[k], g[k], slots["ms"][k], slots["mom"][k], lr)
    elif opt == "gd":
        for k in params:
            newp[k] = apply_gd(params[k], g[k], lr)
    elif opt == "momentum":
        for k in params:
            newp[k], news["accum"][k] = apply_momentum(params[k], g[k], slots["accum"][k], lr)
    elif opt == "adagrad":
        for k in params:
            newp[k], news["accum"][k] = apply_adagrad(params[k], g[k], slots["accum"][k], lr)
    elif opt == "adadelta":
        for k in params:
            newp[k], news["accum"][k], news["accum_update"][k] = apply_adadelta(
                params[k], g[k], slots["accum"][k], slots["accum_update"][k], lr)
    else:
        raise ValueError(opt)
    return newp, news, sc0, g


def init_slots(params, opt="adam", beta1=0.8, beta2=0.75):
    """Optimizer slot initial values as TF-1.2 creates them."""
    z = {k: np.zeros_like(v) for k, v in params.items()}
    if opt == "adam":
        return {"m": z, "v": {k: np.zeros_like(v) for k, v in params.items()},
                "beta1_power": np.float32(beta1), "beta2_power": np.float32(beta2)}
    if opt == "rms":
        return {"ms": {k: np.ones_like(v) for k, v in params.items()}, "mom": z}
    if opt == "momentum":
        return {"accum": z}
    if opt == "adagrad":
        return {"accum": {k: np.full_like(v, 0.1) for k, v in params.items()}}
    if opt == "adadelta":
        return {"accum": z, "accum_update": {k: np.zeros_like(v) for k, v in params.items()}}
    return {}


# --- learner input side: n-step returns (train.py:394-437) and frame history -----------------
#   Pure-Python restatements, pinned by construction to the
# reference's own code paths: the same list operations and numpy calls in the same order.
GAMMA = 0.99                    # train.py:94
LOCAL_TIME_MAX = 5              # train.py:102


def parse_memory(memory, init_r, is_over, gamma=GAMMA):
    """MySimulatorMaster._parse_memory (train.py:418-437).  memory: list of transitions in
    time order, each a dict with 'reward' (Python float) and any payload.  Returns the
    datapoints in queue order as (transition, R, init_r, is_over) with R the float64 value
    the reference computes (R = np.clip(r, -1, 1) + GAMMA * R over the reversed memory) and
    the memory left behind ([last] when not over, [] when over)."""
    mem = list(memory)
    last = None
    if not is_over:
        last = mem[-1]
        mem = mem[:-1]
    mem.reverse()
    R = float(init_r)
    out = []
    for k in mem:
        R = np.clip(k["reward"], -1, 1) + gamma * R
        out.append((k, R, init_r, is_over))
    return out, ([last] if not is_over else [])


class SimulatorMasterMirror(object):
    """The per-client memory logic of SimulatorMaster.run (RL/simulator.py:160-185) with
    MySimulatorMaster's callbacks (train.py:364-437): _on_state appends a transition with the
    predictor's value and the sampled action; the next message sets its reward and then either
    _on_episode_over (parse with init_r = 0) or _on_datapoint (parse when LOCAL_TIME_MAX + 1
    transitions are in memory, bootstrapping from the newest one's value)."""

    def __init__(self, local_time_max=LOCAL_TIME_MAX, gamma=GAMMA):
        self.T = local_time_max + 1
        self.gamma = gamma
        self.memory = {}
        self.queue = []          # datapoints in put order

    def on_message(self, ident, reward, is_over):
        mem = self.memory.setdefault(ident, [])
        if len(mem) > 0:
            mem[-1]["reward"] = reward
            if is_over:
                dps, self.memory[ident] = parse_memory(mem, 0, True, self.gamma)
                self.queue.extend(dps)
            elif len(mem) == self.T:
                dps, self.memory[ident] = parse_memory(mem, mem[-1]["value"], False, self.gamma)
                self.queue.extend(dps)

    def on_state(self, ident, state_id, action, value):
        self.memory.setdefault(ident, []).append(
            {"state": state_id, "action": action, "value": value, "reward": None})


def history_state(frames, hist_len):
    """HistoryFramePlayer.current_state (RL/history.py:29-38): concat of the last hist_len
    frames along the channel axis, zero frames in front while the history is short."""
    hist = list(frames)[-hist_len:]
    pad = [np.zeros_like(hist[0]) for _ in range(hist_len - len(hist))]
    return np.concatenate(pad + hist, axis=2)
