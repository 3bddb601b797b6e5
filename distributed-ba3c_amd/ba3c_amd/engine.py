"""Ba3cEngine — owns the flat parameter / gradient / optimizer-slot buffers (PyTorch-ROCm
device memory) and drives libba3c.so's HIP kernels on the current HIP stream.

This is the MI355X replacement of everything the reference's `sess.run(TfDictOp.op)`
executed per step (tensorpack_cpu/tensorpack/train/trainer.py:282): forward, loss,
autodiff, gradient processor and optimizer apply, plus the predictor's
`sess.run(['towerp0/logitsT','towerp0/pred_value'])` (predict/base.py:80-92).
"""
import ctypes

import numpy as np
import torch

from . import _lib

_F32 = np.float32


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class Ba3cEngine(object):
    """One network instance on one GPU.

    Parameters mirror the reference flag surface: `channels` = FRAME_HISTORY*--channels
    (train.py:95), `fc_neurons` (--fc_neurons), `fc_splits` (--fc_splits),
    `replace_with_conv` (default True; False = --use_normal_fc with `ps` splits).
    """

    def __init__(self, num_actions=4, channels=4, fc_neurons=512, fc_splits=1,
                 replace_with_conv=True, ps=1, max_batch=2048, device=None):
        self.lib = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.Ba3cLibraryError("Ba3cEngine needs a ROCm GPU (torch.cuda unavailable)")
        self.device = torch.device(device or "cuda")
        self.cfg = dict(num_actions=num_actions, channels=channels, fc_neurons=fc_neurons,
                        fc_splits=fc_splits, replace_with_conv=replace_with_conv, ps=ps)
        c = _lib.Ba3cConfig(max_batch, channels, fc_neurons, fc_splits, num_actions,
                            1 if replace_with_conv else 0, ps)
        h = ctypes.c_void_p()
        _lib.check(self.lib.ba3c_create(ctypes.byref(c), ctypes.byref(h)))
        self.h = h
        self.max_batch = max_batch
        self.num_actions = num_actions
        self.channels = channels
        self.layout = []
        for i in range(self.lib.ba3c_num_tensors(h)):
            name = ctypes.c_char_p()
            off, numel = ctypes.c_int64(), ctypes.c_int64()
            shape = (ctypes.c_int32 * 4)()
            nd = ctypes.c_int32()
            _lib.check(self.lib.ba3c_tensor_info(h, i, ctypes.byref(name), ctypes.byref(off),
                                                 ctypes.byref(numel), shape, ctypes.byref(nd)))
            self.layout.append((name.value.decode(), off.value, numel.value,
                                tuple(shape[k] for k in range(nd.value))))
        self.flat_size = int(self.lib.ba3c_flat_size(h))
        with torch.cuda.device(self.device):
            z = lambda: torch.zeros(self.flat_size, dtype=torch.float32, device=self.device)
            self.params = z()
            self.grads = z()
            self.ws_train = None
            self.ws_fwd = None
            self.scalars = torch.zeros(8, dtype=torch.float64, device=self.device)

    # -- parameters -------------------------------------------------------------------
    @property
    def tensor_names(self):
        return [n for n, _, _, _ in self.layout]

    def view(self, flat, name):
        for n, off, numel, shape in self.layout:
            if n == name:
                return flat[off:off + numel].view(shape)
        raise KeyError(name)

    def load_params(self, params):
        """Copy a {name: ndarray} dict (TF layout, e.g. oracle.init_params) into the flat buffer."""
        for n, off, numel, shape in self.layout:
            v = np.ascontiguousarray(params[n], dtype=_F32)
            assert v.shape == shape, (n, v.shape, shape)
            self.params[off:off + numel].copy_(torch.from_numpy(v.reshape(-1)))

    def init_params(self, seed=0, conv_init="normal", fc_init="uniform"):
        """Fresh variables with the reference's initialisers (initializers.py)."""
        from .initializers import initial_values
        self.load_params(initial_values(self.layout, seed=seed, conv_init=conv_init,
                                        fc_init=fc_init,
                                        replace_with_conv=self.cfg["replace_with_conv"]))

    def state_dict(self, flat=None):
        flat = self.params if flat is None else flat
        host = flat.detach().cpu().numpy()
        return {n: host[off:off + numel].reshape(shape).copy() for n, off, numel, shape in self.layout}

    def zeros_like_flat(self, fill=0.0):
        return torch.full((self.flat_size,), fill, dtype=torch.float32, device=self.device)

    # -- workspaces ---------------------------------------------------------------------
    def _workspace(self, train):
        if train:
            if self.ws_train is None:
                n = self.lib.ba3c_workspace_size(self.h, self.max_batch, 1)
                self.ws_train = torch.empty(n, dtype=torch.uint8, device=self.device)
            return self.ws_train
        if self.ws_fwd is None:
            n = self.lib.ba3c_workspace_size(self.h, self.max_batch, 0)
            self.ws_fwd = torch.empty(n, dtype=torch.uint8, device=self.device)
        return self.ws_fwd

    def workspace_tensor(self, name, batch, train=True):
        """View of an intermediate of the last call with this batch (tests / debugging)."""
        off, nb = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self.lib.ba3c_workspace_tensor(self.h, batch, 1 if train else 0,
                                                  name.encode(), ctypes.byref(off),
                                                  ctypes.byref(nb)))
        ws = self._workspace(train)
        raw = ws[off.value:off.value + nb.value]
        return raw if name.startswith("c") else raw.view(torch.float32)

    def _check_state(self, state):
        assert state.dtype == torch.uint8 and state.is_cuda and state.is_contiguous(), \
            "state must be a contiguous uint8 device tensor [B,84,84,C]"
        assert state.dim() == 4 and tuple(state.shape[1:]) == (84, 84, self.channels), state.shape
        B = state.shape[0]
        assert 1 <= B <= self.max_batch, "batch %d outside [1, %d]" % (B, self.max_batch)
        return B

    # -- hot path -------------------------------------------------------------------------
    def forward(self, state, explore_factor=1.0, params=None, out=None):
        """Predictor forward: returns (probs 'logits', probsT 'logitsT', value 'pred_value')."""
        B = self._check_state(state)
        A = self.num_actions
        if out is None:
            out = (torch.empty(B, A, dtype=torch.float32, device=self.device),
                   torch.empty(B, A, dtype=torch.float32, device=self.device),
                   torch.empty(B, dtype=torch.float32, device=self.device))
        params = self.params if params is None else params
        _lib.check(self.lib.ba3c_forward(self.h, _stream(), _ptr(params), _ptr(state), B,
                                         float(explore_factor), _ptr(self._workspace(False)),
                                         _ptr(out[0]), _ptr(out[1]), _ptr(out[2])))
        return out

    def train_grads(self, state, action, futurereward, entropy_beta=0.01, grads=None, phase=0):
        """Forward + loss + backward; raw gradients into `grads` (default self.grads).
        Returns the device float64 scalars tensor (order: _lib.SCALAR_NAMES).  phase 1 / 2
        split the pass at the fc1 + heads bucket (ba3c_train_grads_phase); phase 3 leaves the
        final gradient reduction to the next fused-clip apply_update (one launch fewer): until
        then `grads` holds unreduced data for any reader outside this handle — call
        flush_pending() before reading it through torch."""
        B = self._check_state(state)
        assert action.dtype == torch.int64 and action.shape == (B,) and action.is_cuda
        assert futurereward.dtype == torch.float32 and futurereward.shape == (B,)
        grads = self.grads if grads is None else grads
        _lib.check(self.lib.ba3c_train_grads_phase(self.h, _stream(), _ptr(self.params), _ptr(state),
                                                   _ptr(action.contiguous()),
                                                   _ptr(futurereward.contiguous()), B,
                                                   float(entropy_beta), _ptr(self._workspace(True)),
                                                   _ptr(grads), _ptr(self.scalars), int(phase)))
        return self.scalars

    def flush_pending(self):
        """Launch a weight-gradient reduction a phase-3 pass left pending (no-op otherwise)."""
        _lib.check(self.lib.ba3c_flush_pending(self.h))

    def occupy_cus(self, stream, n_cus, usec):
        """Diagnostic: hold `n_cus` CUs for `usec` microseconds on torch stream `stream`."""
        _lib.check(self.lib.ba3c_occupy_cus(ctypes.c_void_p(stream.cuda_stream), int(n_cus),
                                            float(usec)))

    def bucket_split(self):
        """(first tensor, flat offset) of the fc1 + heads gradient bucket."""
        t = int(self.lib.ba3c_bucket_tensor(self.h))
        return t, self.layout[t][1]

    def clip_grads_range(self, t0, t1, grads=None, no_residency=False):
        """clip_by_average_norm over tensors [t0, t1) only.  no_residency: the two-launch form
        (for a stream that runs beside other kernels, ba3c_clip_grads_range2)."""
        grads = self.grads if grads is None else grads
        _lib.check(self.lib.ba3c_clip_grads_range2(self.h, _stream(), _ptr(grads),
                                                   _ptr(self._workspace(True)), int(t0), int(t1),
                                                   1 if no_residency else 0))

    def launch_held(self, stream=None):
        """Launch the fc1 + heads reduction a phase-4 pass held back, on `stream` (a torch
        stream, default the current one), ordered after the pass's stream."""
        st = ctypes.c_void_p((stream or torch.cuda.current_stream()).cuda_stream)
        _lib.check(self.lib.ba3c_launch_held(self.h, st))

    def set_phase2_event(self, event):
        """Record `event` (a hipevent.HipEvent, or None) after conv3's gradient launches of every
        later phase-2 pass."""
        _lib.check(self.lib.ba3c_set_phase2_event(self.h, event._ev if event is not None else None))

    def clip_grads(self, grads=None):
        """tf.clip_by_average_norm(g, 0.1) per tensor, in place (train.py:329-330)."""
        grads = self.grads if grads is None else grads
        _lib.check(self.lib.ba3c_clip_grads(self.h, _stream(), _ptr(grads),
                                            _ptr(self._workspace(True))))

    def apply_update(self, opt, slot0, slot1, hp, grad_scale=1.0, fuse_clip=False, grads=None,
                     dev_powers=None):
        """One optimizer apply; dev_powers (float32 device tensor [2]) keeps Adam's
        beta-power state on the GPU (required inside a captured hipGraph)."""
        grads = self.grads if grads is None else grads
        p = _lib.Ba3cOptParams(**hp)
        if dev_powers is None:
            _lib.check(self.lib.ba3c_apply_update(self.h, _stream(), _lib.OPT_IDS[opt],
                                                  _ptr(self.params), _ptr(grads), _ptr(slot0),
                                                  _ptr(slot1), ctypes.byref(p), float(grad_scale),
                                                  1 if fuse_clip else 0,
                                                  _ptr(self._workspace(True))))
        else:
            _lib.check(self.lib.ba3c_apply_update_dev(self.h, _stream(), _lib.OPT_IDS[opt],
                                                      _ptr(self.params), _ptr(grads), _ptr(slot0),
                                                      _ptr(slot1), ctypes.byref(p), _ptr(dev_powers),
                                                      float(grad_scale), 1 if fuse_clip else 0,
                                                      _ptr(self._workspace(True))))

    def sample(self, probs, u, actions=None, flag=None):
        """numpy RandomState.choice(A, p) given the uniform draws u (float64 device tensor)."""
        B, A = probs.shape
        assert u.dtype == torch.float64 and u.shape == (B,)
        if actions is None:
            actions = torch.empty(B, dtype=torch.int64, device=probs.device)
        if flag is None:
            flag = torch.zeros(1, dtype=torch.int32, device=probs.device)
        _lib.check(self.lib.ba3c_sample(_stream(), _ptr(probs.contiguous()), _ptr(u), B, A,
                                        _ptr(actions), _ptr(flag)))
        return actions, flag

    def greedy(self, probs, u, random_actions, eps=0.001, actions=None):
        """Evaluation action: first argmax of each row, random_actions[i] where u[i] < eps."""
        B, A = probs.shape
        assert u.dtype == torch.float64 and u.shape == (B,)
        assert random_actions.dtype == torch.int64 and random_actions.shape == (B,)
        if actions is None:
            actions = torch.empty(B, dtype=torch.int64, device=probs.device)
        _lib.check(self.lib.ba3c_greedy(_stream(), _ptr(probs.contiguous()), _ptr(u),
                                        _ptr(random_actions.contiguous()), B, A, float(eps),
                                        _ptr(actions)))
        return actions

    # -- timing probe -------------------------------------------------------------------
    def probe_enable(self, kernel, every=1):
        """Bracket launches of `kernel` (None: stop) with HIP events, the first of every
        `every` of them (ba3c_probe_every)."""
        kid = -1 if kernel is None else _lib.KERNEL_IDS[kernel]
        _lib.check(self.lib.ba3c_probe_enable(self.h, kid))
        if every != 1 or hasattr(self.lib, "ba3c_probe_every"):   # (A/B builds predating it)
            _lib.check(self.lib.ba3c_probe_every(self.h, int(every)))

    def kernel_merged(self, kernel):
        """Kernel names that ran inside `kernel`'s launch in the last training pass (multi-job
        launches; ba3c_kernel_merged)."""
        if not hasattr(self.lib, "ba3c_kernel_merged"):
            return []
        m = int(self.lib.ba3c_kernel_merged(self.h, _lib.KERNEL_IDS[kernel]))
        return [] if m <= 0 else [k for k, i in _lib.KERNEL_IDS.items() if m >> i & 1]

    def kernel_split(self, kernel):
        """16-bit MFMA products per fp32 product of `kernel` on this handle (6: bf16 hi/mid/lo,
        3: scaled fp16 hi/lo or conv0's u8 x bf16x3, 2: conv0's u8 x fp16 hi/lo, 1: fp32 MFMA,
        0: no matrix work)."""
        return int(self.lib.ba3c_kernel_split(self.h, _lib.KERNEL_IDS[kernel]))

    def kernel_family(self, kernel):
        """3: bf16 split planes, 2: scaled fp16 split planes, else kernel_split's value."""
        return int(self.lib.ba3c_kernel_family(self.h, _lib.KERNEL_IDS[kernel]))

    def device_errors(self):
        """Error flags of the handle's in-launch waits (0 = none; synchronises the device)."""
        f = ctypes.c_uint32()
        _lib.check(self.lib.ba3c_device_errors(self.h, ctypes.byref(f)))
        return f.value

    def probe_read(self):
        ms, n = ctypes.c_double(), ctypes.c_int32()
        _lib.check(self.lib.ba3c_probe_read(self.h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.lib.ba3c_destroy(self.h)
                self.h = None
        except Exception:
            pass
