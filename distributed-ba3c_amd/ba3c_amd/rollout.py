"""The learner's input side on the GPU.

`RolloutBuffer` is MySimulatorMaster's per-client memory (OpenAIGym/train.py:364-437,
RL/simulator.py:160-185) for a vector of simulators, kept in HBM: `on_state` appends each
simulator's new transition (state, sampled action, predictor value) as `_on_state` does,
`on_reward` sets the newest transition's reward and — for every simulator whose episode ended
or whose memory holds LOCAL_TIME_MAX + 1 transitions — runs `_parse_memory` on the GPU
(`ba3c_nstep_returns`), gathering the emitted datapoints' states and actions
(`ba3c_gather_rows`) before their ring slots are reused.  `BatchQueue` is BatchData(B) over the
datapoint stream (dataflow/common.py:64-99) without the host queue of EnqueueThread
(train/trainer.py:116-155).  `FrameHistory` is HistoryFramePlayer (RL/history.py:12-55) on
the device (`ba3c_history_push`).

Ordering matches the reference: datapoints of one parse come env by env, each env's in the
reverse time order `_parse_memory` puts them on its queue.
"""
import ctypes

import numpy as np
import torch

from . import _lib

GAMMA = 0.99              # train.py:94
LOCAL_TIME_MAX = 5        # train.py:102
IMAGE_SIZE = (84, 84)     # train.py:92


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class Datapoints(object):
    """One parse's datapoints: [state, action, R, init_R, isOver] (train.py:432; the ts field
    is carried separately by callers that track it)."""

    def __init__(self, state, action, R, init_R, over, src):
        self.state, self.action, self.R, self.init_R, self.over, self.src = \
            state, action, R, init_R, over, src

    def __len__(self):
        return int(self.R.shape[0])


class RolloutBuffer(object):
    def __init__(self, n_envs, channels=4, local_time_max=LOCAL_TIME_MAX, gamma=GAMMA,
                 device="cuda"):
        self.lib = _lib.load()
        self.E, self.T = int(n_envs), int(local_time_max) + 1
        self.C = int(channels)
        self.gamma = float(gamma)
        dev = torch.device(device)
        self.device = dev
        E, T = self.E, self.T
        self.states = torch.zeros((E, T) + IMAGE_SIZE + (self.C,), dtype=torch.uint8, device=dev)
        self.actions = torch.zeros(E, T, dtype=torch.int64, device=dev)
        self.values = torch.zeros(E, T, dtype=torch.float32, device=dev)
        self.rewards = torch.zeros(E, T, dtype=torch.float64, device=dev)
        self.start = torch.zeros(E, dtype=torch.int32, device=dev)
        self.length = torch.zeros(E, dtype=torch.int32, device=dev)
        # scratch of one parse
        n = E * T
        self._R = torch.empty(n, dtype=torch.float32, device=dev)
        self._src = torch.empty(n, dtype=torch.int32, device=dev)
        self._init = torch.empty(n, dtype=torch.float32, device=dev)
        self._over = torch.empty(n, dtype=torch.uint8, device=dev)
        self._count = torch.zeros(1, dtype=torch.int32, device=dev)
        self._ar = torch.arange(E, device=dev, dtype=torch.int64)

    def _slot(self, offset):
        return ((self.start + self.length + offset) % self.T).long()

    def on_state(self, states, actions, values):
        """_on_state (train.py:364-392) for every simulator: append (state, action, value)."""
        assert states.shape == (self.E,) + IMAGE_SIZE + (self.C,) and states.dtype == torch.uint8
        slot = self._slot(0)
        self.states[self._ar, slot] = states
        self.actions[self._ar, slot] = actions.to(torch.int64)
        self.values[self._ar, slot] = values.to(torch.float32)
        self.length += 1

    def on_reward(self, rewards, is_over):
        """SimulatorMaster.run's `memory[-1].reward = reward` followed by _on_episode_over /
        _on_datapoint for every simulator (train.py:394-416).  Returns the Datapoints emitted."""
        has = self.length > 0
        slot = self._slot(-1)
        r = rewards.to(device=self.device, dtype=torch.float64)
        self.rewards[self._ar, slot] = torch.where(has, r, self.rewards[self._ar, slot])
        over = is_over.to(device=self.device, dtype=torch.bool) & has
        ready = over | (self.length == self.T)
        plen = torch.where(ready, self.length, torch.zeros_like(self.length))
        over_u8 = over.to(torch.uint8)
        _lib.check(self.lib.ba3c_nstep_returns(
            _stream(), _ptr(self.rewards), _ptr(self.values), _ptr(self.start), _ptr(plen),
            _ptr(over_u8), self.E, self.T, ctypes.c_double(self.gamma), _ptr(self._R),
            _ptr(self._src), _ptr(self._init), _ptr(self._over), _ptr(self._count)))
        n = int(self._count.item())
        out = self._gather(n)
        # memory left behind: [last] when not over, [] when over
        keep_last = ready & ~over
        self.start = torch.where(over, (self.start + self.length) % self.T,
                                 torch.where(keep_last, (self.start + self.length - 1) % self.T,
                                             self.start)).to(torch.int32)
        self.length = torch.where(over, torch.zeros_like(self.length),
                                  torch.where(keep_last, torch.ones_like(self.length),
                                              self.length)).to(torch.int32)
        return out

    def _gather(self, n):
        src = self._src[:n].clone()
        st = torch.empty((n,) + IMAGE_SIZE + (self.C,), dtype=torch.uint8, device=self.device)
        ac = torch.empty(n, dtype=torch.int64, device=self.device)
        row = IMAGE_SIZE[0] * IMAGE_SIZE[1] * self.C
        if n == 0:
            return Datapoints(st, ac, self._R[:0].clone(), self._init[:0].clone(),
                              self._over[:0].clone(), src)
        _lib.check(self.lib.ba3c_gather_rows(_stream(), _ptr(self.states), _ptr(src), n, row, _ptr(st)))
        _lib.check(self.lib.ba3c_gather_rows(_stream(), _ptr(self.actions), _ptr(src), n, 8, _ptr(ac)))
        return Datapoints(st, ac, self._R[:n].clone(), self._init[:n].clone(),
                          self._over[:n].clone(), src)


class BatchQueue(object):
    """BatchData(B) over the datapoint stream (dataflow/common.py:64-99): batches of exactly
    B datapoints in arrival order; the remainder waits for the next parse."""

    def __init__(self, batch_size):
        self.B = int(batch_size)
        self._parts = []
        self._n = 0

    def put(self, dps):
        if len(dps):
            self._parts.append(dps)
            self._n += len(dps)

    def __len__(self):
        return self._n

    def get(self):
        """Next [state, action, futurereward, init_R, isOver] batch, or None."""
        if self._n < self.B:
            return None
        cat = lambda name: torch.cat([getattr(p, name) for p in self._parts])
        fields = [cat(k) for k in ("state", "action", "R", "init_R", "over", "src")]
        B = self.B
        batch = [f[:B] for f in fields]
        rest = Datapoints(*[f[B:] for f in fields])
        self._parts = [rest] if len(rest) else []
        self._n = len(rest)
        return batch[:5]


class FrameHistory(object):
    """HistoryFramePlayer(player, FRAME_HISTORY) for a vector of simulators (train.py:124,
    RL/history.py:12-55): `state` [E,84,84,hist_len*c] uint8 on the device."""

    def __init__(self, n_envs, hist_len=4, channels=1, device="cuda"):
        self.lib = _lib.load()
        self.E, self.H, self.c = int(n_envs), int(hist_len), int(channels)
        self.state = torch.zeros((self.E,) + IMAGE_SIZE + (self.H * self.c,), dtype=torch.uint8,
                                 device=device)

    def push(self, frames, is_over=None):
        """Append one frame per simulator; is_over[e] = the frame starts a new episode."""
        assert frames.dtype == torch.uint8 and frames.is_contiguous()
        ov = None if is_over is None else is_over.to(torch.uint8).contiguous()
        _lib.check(self.lib.ba3c_history_push(_stream(), _ptr(frames), _ptr(self.state), _ptr(ov),
                                              self.E, IMAGE_SIZE[0] * IMAGE_SIZE[1], self.H, self.c))
        return self.state
