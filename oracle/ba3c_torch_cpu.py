"""PyTorch-CPU fp32 restatement of the reference TF-1.2 train step — TEST / BASELINE
INFRASTRUCTURE ONLY (bench.py's `cpu_baseline` leg and tests/ may use it; the product path
never does).

This is the "CPU restatement of the reference TF graph" that SURVEY.md §8d / BASELINE.md §2
ask to time beside the GPU: the same ops as `OpenAIGym/train.py:164-330` and `:582-597`
(16-channel zero padding :173-174, conv/ReLU/max-pool tower :177-212, FC1 as S 5x5 VALID convs
with no bias and no ReLU :216-229, heads :250-264, softmax / log(p+1e-6) / A3C loss :286-327,
autodiff, per-tensor clip_by_average_norm(0.1) :329-330, TF ApplyAdam with float32 beta powers)
on torch's CPU kernels in float32 — the arithmetic type of the reference.
Its numerics are checked against the numpy oracle in tests/test_oracle.py.  The convolutions
run with oneDNN disabled (torch's im2col + MKL GEMM path): oneDNN's fp32 weight gradient of
conv0 came out 1.8e-2 (relative to max|g|) off the fp64 oracle on a 3-frame case where the
im2col path is within 1.3e-6, and a baseline must compute the reference's step, not a faster
wrong one.
"""
import torch
import torch.nn.functional as Fn

TARGET_CHANNELS = 16


class TorchCpuBa3c(object):
    def __init__(self, params, fc_neurons, fc_splits, lr=1e-3, beta1=0.8, beta2=0.75, eps=1e-8,
                 entropy_beta=0.01):
        """params: {name: float32 ndarray} in TF layout (oracle.init_params)."""
        self.F, self.S = fc_neurons, fc_splits
        self.names = list(params)
        self.p = {k: torch.tensor(v, dtype=torch.float32) for k, v in params.items()}
        self.m = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps
        self.b1p = torch.tensor(beta1, dtype=torch.float32)
        self.b2p = torch.tensor(beta2, dtype=torch.float32)
        self.beta = entropy_beta

    def _forward(self, w, state):
        """train.py:164-299 on NHWC uint8 frames; returns (probs, value, flat-free extras)."""
        B, _, _, C = state.shape
        x = state.to(torch.float32) / 255.0                                      # :167
        x = torch.cat([x, torch.zeros(B, 84, 84, TARGET_CHANNELS - C)], dim=3)     # :173-174
        x = x.permute(0, 3, 1, 2)                                                # NCHW view

        def conv(x, W):                   # HWIO -> OIHW
            return Fn.conv2d(x, W.permute(3, 2, 0, 1))
        x = Fn.max_pool2d(Fn.relu(conv(x, w["conv0/W"])), 2)                      # :177-185
        x = Fn.max_pool2d(Fn.relu(conv(x, w["conv1/W"])), 2)                      # :187-195
        x = Fn.max_pool2d(Fn.relu(conv(x, w["conv2/W"])), 2)                      # :197-204
        x = Fn.relu(conv(x, w["conv3/W"]))                                        # :206-207
        flat = x.permute(0, 2, 3, 1).reshape(B, 1600)                            # NHWC flatten
        per = self.F // self.S
        W1 = torch.cat([w["fc1_%d/W" % i].reshape(1600, per) for i in range(self.S)], dim=1)
        h = flat @ W1                                                            # :216-229
        policy = h @ w["fc-pi/W"] + w["fc-pi/b"]                                 # :250-252
        value = (h @ w["fc-v/W"] + w["fc-v/b"])[:, 0]                            # :257-259
        return torch.softmax(policy, dim=1), value

    def loss_and_grads(self, state, action, R):
        with torch.backends.mkldnn.flags(enabled=False), torch.enable_grad():
            return self._loss_and_grads(state, action, R)

    def _loss_and_grads(self, state, action, R):
        w = {k: v.detach().requires_grad_(True) for k, v in self.p.items()}
        p, V = self._forward(w, state)
        B = float(state.shape[0])
        logp = torch.log(p + 1e-6)                                               # :305
        lpa = logp.gather(1, action[:, None])[:, 0]
        adv = V.detach() - R                                                     # :309
        cost = ((lpa * adv).sum() + self.beta * (p * logp).sum()
                + ((V - R) ** 2).sum() / 2.0) / B                                # :310-327
        grads = torch.autograd.grad(cost, [w[k] for k in self.names])
        return cost.detach(), dict(zip(self.names, grads))

    @torch.no_grad()
    def step(self, state, action, R):
        """One sess.run(TfDictOp.op): forward, loss, backward, clip, Adam."""
        cost, g = self.loss_and_grads(state, action, R)
        alpha = self.lr * torch.sqrt(1.0 - self.b2p) / (1.0 - self.b1p)
        for k in self.names:
            t = g[k]
            n = float(t.numel())
            ss = (t * t).sum()
            mult = torch.clamp(torch.rsqrt(ss) * n, max=10.0)                    # :329-330
            t = (t * 0.1) * mult
            m, v = self.m[k], self.v[k]
            m += (t - m) * (1.0 - self.b1)
            v += (t * t - v) * (1.0 - self.b2)
            self.p[k] -= (m * alpha) / (torch.sqrt(v) + self.eps)
        self.b1p *= self.b1
        self.b2p *= self.b2
        return cost
