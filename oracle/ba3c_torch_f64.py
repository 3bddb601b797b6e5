"""Float64 PyTorch restatement of the reference TF-1.2 forward + loss + backward, driven by a
checked implementation's own discrete decisions — TEST INFRASTRUCTURE ONLY (tests/ use it as
the checker; the product path never imports it).

Why it exists: the numpy oracle (`ba3c_oracle.loss_and_grads_chunked`) needs ~10 s per 128
samples, too slow for the bench workload itself (B=2048, F=512).  This module computes the same
function — `OpenAIGym/train.py:164-327` differentiated as `train/multigpu.py:85-86` does — with
torch's float64 convolutions and autograd on the CPU (the B=2048 GPU test runs it on the
host as the checker, ~20 s: an implementation independent of the HIP kernels).  It is pinned to the numpy oracle by `tests/test_oracle.py` (same forced decisions,
agreement ~1e-12 at small B).

Forced decisions (`forced`, as `ba3c_oracle.loss_and_grads(forced=...)`): the max-pool argmax
code of every window (`c0`..`c2`, 0..3 = row-major position of the first maximum, 255 = window
max <= 0, i.e. ReLU gradient 0) and conv3's ReLU mask (`a3_mask`).  The pooled value is the
pre-activation at the forced position (0 for code 255), so forward and backward follow the
checked side's decisions; a decision differs from fp64's own only on fp32 near-ties, where the
two candidate values agree to rounding.

Only the real input channels are convolved: the 12 zero channels of the 16-channel padding
(`train.py:173-174`) contribute nothing to any output, and their weight gradient is exactly zero
(appended as zeros, so `conv0/W`'s gradient keeps the graph's [5,5,16,32] shape).
"""
import numpy as np
import torch
import torch.nn.functional as Fn

TARGET_CHANNELS = 16
LOG_EPS = 1e-6                 # train.py:305


def _pool_forced(z, code):
    """z: [B,C,H,W] pre-activation; code: [B,H/2,W/2,C] uint8 (NHWC, as the workspace holds it).
    Returns the pooled map [B,C,H/2,W/2]: z at the forced window position, 0 for code 255."""
    B, C, H, W = z.shape
    win = z.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(
        B, C, H // 2, W // 2, 4)
    c = code.permute(0, 3, 1, 2).to(torch.int64)                # [B,C,H/2,W/2]
    dead = c == 255
    p = torch.gather(win, 4, torch.where(dead, 0, c)[..., None])[..., 0]
    return torch.where(dead, torch.zeros_like(p), p)


def own_decisions(params, state, chunk=256, device="cpu", tol=2e-5):
    """The float64 forward's own discrete decisions (`ba3c_oracle.maxpool2x2_argmax`: first
    maximum in row-major window order, code 255 where the window max <= 0; conv3's ReLU mask),
    in the workspace's NHWC layouts — to count how often a checked side decided otherwise —
    and where those decisions are numerically ambiguous (`near_c0`..`near_c2`, `near_a3`:
    `ba3c_oracle.ambiguous_windows` / `ambiguous_relu` — a competitor not exactly equal to
    the window max but within tol x the image's max |z| of it, or a max / pre-activation that
    close to zero without being zero)."""
    dev = torch.device(device)
    C = state.shape[3]
    W = {k: torch.tensor(np.asarray(params[k], np.float64), device=dev).permute(3, 2, 0, 1)
         for k in ("conv0/W", "conv1/W", "conv2/W", "conv3/W")}
    W["conv0/W"] = W["conv0/W"][:, :C]
    out = {k: [] for k in ("c0", "c1", "c2", "a3_mask", "near_c0", "near_c1", "near_c2",
                           "near_a3")}

    def image_eps(z):
        return tol * z.abs().reshape(z.shape[0], -1).max(dim=1).values.reshape(-1, 1, 1, 1)

    def pool(z):
        B, Cc, H, Wd = z.shape
        win = z.reshape(B, Cc, H // 2, 2, Wd // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(
            B, Cc, H // 2, Wd // 2, 4)
        mx, code = win.max(dim=4)           # first maximum (torch returns the first index)
        eps = image_eps(z)
        gap = mx[..., None] - win
        near = ((gap > 0) & (gap <= eps[..., None])).any(dim=4) | \
            ((mx != 0) & (mx.abs() <= eps))
        code = torch.where(mx > 0, code, 255).to(torch.uint8)
        return torch.relu(mx), code.permute(0, 2, 3, 1), near.permute(0, 2, 3, 1)
    with torch.no_grad():
        for lo in range(0, state.shape[0], chunk):
            x = torch.as_tensor(state[lo:lo + chunk], device=dev).to(torch.float64) / 255.0
            p = x.permute(0, 3, 1, 2)
            for i in range(3):
                p, c, near = pool(Fn.conv2d(p, W["conv%d/W" % i]))
                out["c%d" % i].append(c.cpu().numpy())
                out["near_c%d" % i].append(near.cpu().numpy())
            z3 = Fn.conv2d(p, W["conv3/W"])
            out["a3_mask"].append((z3 > 0).permute(0, 2, 3, 1).cpu().numpy())
            near3 = (z3 != 0) & (z3.abs() <= image_eps(z3))
            out["near_a3"].append(near3.permute(0, 2, 3, 1).cpu().numpy())
    return {k: np.concatenate(v) for k, v in out.items()}


def loss_and_grads_forced(params, state, action, futurereward, cfg, forced, entropy_beta=0.01,
                          device="cpu", chunk=None):
    """Float64 gradients of `cost` (train.py:326-327) w.r.t. every trainable variable, with the
    backward pass routed by `forced`.  params: {name: ndarray} TF layouts; state uint8
    [B,84,84,C]; returns ({name: float64 ndarray}, {'cost', 'pred_value', 'logits'}).
    `chunk` evaluates the batch in sub-batches (the cost is a batch mean, so the gradient is the
    B_c/B-weighted sum of the chunks' gradients)."""
    assert cfg.get("replace_with_conv", True), "identity FC (the default FC) only"
    B = state.shape[0]
    chunk = chunk or B
    dev = torch.device(device)
    names = list(params)
    w = {k: torch.tensor(np.asarray(v, np.float64), device=dev) for k, v in params.items()}
    C = state.shape[3]
    F, S = cfg["fc_neurons"], cfg.get("fc_splits", 1)
    per = F // S
    acc = {k: torch.zeros_like(v) for k, v in w.items()}
    cost_total = 0.0
    probs, values = [], []
    for lo in range(0, B, chunk):
        hi = min(B, lo + chunk)
        ww = {k: v.detach().clone().requires_grad_(True) for k, v in w.items()}
        x = torch.as_tensor(state[lo:hi], device=dev).to(torch.float64) / 255.0   # :167
        x = x.permute(0, 3, 1, 2)
        fc = {k: torch.as_tensor(np.ascontiguousarray(forced[k][lo:hi]), device=dev)
              for k in ("c0", "c1", "c2")}

        def conv(x, W):                    # HWIO -> OIHW, VALID, stride 1 (conv2d.py:63-66)
            return Fn.conv2d(x, W.permute(3, 2, 0, 1))
        W0 = ww["conv0/W"][:, :, :C, :]                                          # real channels
        p = _pool_forced(conv(x, W0), fc["c0"])                                  # :177-185
        p = _pool_forced(conv(p, ww["conv1/W"]), fc["c1"])                       # :187-195
        p = _pool_forced(conv(p, ww["conv2/W"]), fc["c2"])                       # :197-204
        m3 = torch.as_tensor(np.ascontiguousarray(forced["a3_mask"][lo:hi]), device=dev)
        a3 = conv(p, ww["conv3/W"]) * m3.permute(0, 3, 1, 2).to(torch.float64)   # :206-207
        flat = a3.permute(0, 2, 3, 1).reshape(hi - lo, 1600)                     # NHWC flatten
        W1 = torch.cat([ww["fc1_%d/W" % i].reshape(1600, per) for i in range(S)], dim=1)
        h = flat @ W1                                                            # :216-229
        policy = h @ ww["fc-pi/W"] + ww["fc-pi/b"]                               # :250-252
        V = (h @ ww["fc-v/W"] + ww["fc-v/b"])[:, 0]                              # :257-259
        pr = torch.softmax(policy, dim=1)                                        # :288
        R = torch.as_tensor(np.asarray(futurereward[lo:hi], np.float64), device=dev)
        a = torch.as_tensor(np.asarray(action[lo:hi], np.int64), device=dev)
        logp = torch.log(pr + LOG_EPS)                                           # :305
        lpa = logp.gather(1, a[:, None])[:, 0]                                   # :307-308
        adv = V.detach() - R                                                     # :309
        cost = ((lpa * adv).sum() + entropy_beta * (pr * logp).sum()
                + ((V - R) ** 2).sum() / 2.0) / float(B)                         # :310-327
        g = torch.autograd.grad(cost, [ww[k] for k in names], allow_unused=True)
        for k, gk in zip(names, g):
            if gk is not None:
                acc[k] += gk
        cost_total += float(cost.detach())
        probs.append(pr.detach().cpu().numpy())
        values.append(V.detach().cpu().numpy())
    grads = {k: v.cpu().numpy() for k, v in acc.items()}
    return grads, {"cost": cost_total, "logits": np.concatenate(probs),
                   "pred_value": np.concatenate(values)}
