"""Learner step driver: QueueInputTrainer.run_step / AsyncMultiGPUTrainer.run_step
(train/trainer.py:244-299, train/multigpu.py:131-324) re-designed for one process per GPU.

One `run_step(batch)` = forward + A3C loss + backward (one HIP launch chain), the model's
gradient processors (fused clip), the synchronous RCCL gradient mean when
SyncReplicasOptimizer is used, and one fused optimizer apply; it returns the TfDictOp
dictionary of the reference (multigpu.py:193-205).
"""
import os
import time

import numpy as np
import torch

from .model_desc import ClipByAverageNorm, MapGradient
from . import hipevent
from .optimizer import SyncReplicasOptimizer


class TrainConfig(object):
    """train/config.py:15-84 (the fields this path uses)."""

    def __init__(self, model, optimizer, dataset=None, step_per_epoch=250, max_epoch=1000,
                 callbacks=None, extra_arg=None):
        self.model = model
        self.optimizer = optimizer
        self.dataset = dataset
        self.step_per_epoch = step_per_epoch
        self.max_epoch = max_epoch
        self.callbacks = callbacks or []
        self.extra_arg = extra_arg or {}


class ExchangeTimeline(object):
    """HIP timing events of the bucketed data-parallel step (Ba3cTrainer._bucketed_sync_step),
    recorded inside the real step: on the learner stream `start`, `phase1_end`, `conv_ready`
    (phase 2 + the conv bucket's clip done), `exchanged` (both sums joined) and `end` (update
    applied); on the exchange stream `fc1_start` (the phase-2 event passed), `fc1_ready` (the
    held fc1 + heads reduction and the bucket's clip done) and each bucket's all-reduce
    begin / end.  summary() averages the intervals over the steps."""

    MAIN = ("start", "phase1_end", "conv_ready", "exchanged", "end")
    COMM = ("fc1_start", "fc1_ready", "fc1_ar_begin", "fc1_ar_end", "conv_ar_begin", "conv_ar_end")

    def __init__(self):
        self.steps = []

    def new_step(self):
        ev = {k: hipevent.timing_event() for k in self.MAIN + self.COMM}
        self.steps.append(ev)
        return ev

    def summary(self):
        """Mean milliseconds of each interval (call after the device has synchronised)."""
        if not self.steps:
            return None
        keys = {"phase1_ms": ("start", "phase1_end"), "phase2_ms": ("phase1_end", "conv_ready"),
                # exchange stream: the held fc1 + heads reduction and the bucket's clip, from
                # the phase-2 event (after conv3) on
                "fc1_prep_ms": ("fc1_start", "fc1_ready"),
                "fc1_start_after_phase1_ms": ("phase1_end", "fc1_start"),
                "fc1_allreduce_ms": ("fc1_ar_begin", "fc1_ar_end"),
                "conv_allreduce_ms": ("conv_ar_begin", "conv_ar_end"),
                "exposed_ms": ("conv_ready", "exchanged"), "update_ms": ("exchanged", "end"),
                "step_ms": ("start", "end"),
                # > 0: the fc1 + heads sum outlasted the conv backward by this much
                "fc1_allreduce_tail_ms": ("conv_ready", "fc1_ar_end")}
        out = {}
        for name, (a, b) in keys.items():
            out[name] = round(float(np.mean([s[a].elapsed_time(s[b]) for s in self.steps])), 4)
        out["steps"] = len(self.steps)
        return out


class Ba3cTrainer(object):
    def __init__(self, config):
        self.config = config
        self.model = config.model
        self.engine = config.model.engine
        self.optimizer = config.optimizer
        self.global_step = 0
        self.step_ms = []
        procs = self.model.get_gradient_processor()
        self._fused_clip = (len(procs) == 1 and isinstance(procs[0], MapGradient)
                            and isinstance(procs[0].func, ClipByAverageNorm)
                            and procs[0].regex == ".*$")
        self._procs = procs
        # BA3C_DEFER_REDUCE=1 (single replica): the pass's weight-gradient reduction rides on the
        # fused apply's launch (ba3c_train_grads_phase phase 3: one launch fewer).  Default off:
        # same-box r05ab, B=32 step 0.1607 -> 0.1646 ms, B=2048 1.743 -> 1.752 ms (the hand-off's
        # agent-scope stores / loads and signal counters cost more than the launch boundary)
        flag = os.environ.get("BA3C_DEFER_REDUCE", "0")
        if flag not in ("0", "1"):
            raise ValueError("BA3C_DEFER_REDUCE must be 0 or 1 (got %r)" % flag)
        self._defer_reduce = flag == "1"
        # BA3C_XCHG_HELD=1: the N>1 step holds phase 1's fc1 + heads reduction and runs it and
        # the bucket's clip on the exchange stream (ba3c_launch_held).  Default 0: same-box
        # r06c, the held work beside conv2's launch stretched that launch by 24 us, more than
        # the ~16 us it took off the learner stream
        flag = os.environ.get("BA3C_XCHG_HELD", "0")
        if flag not in ("0", "1"):
            raise ValueError("BA3C_XCHG_HELD must be 0 or 1 (got %r)" % flag)
        self._xchg_held = flag == "1"
        if isinstance(self.optimizer, SyncReplicasOptimizer):
            self.optimizer.broadcast_variables(self.engine)

    def process_grads(self):
        for p in self._procs:
            p.process(self.engine)

    @staticmethod
    def describe_device_errors(flags):
        """Decode ba3c_device_errors' bits (include/ba3c.h)."""
        what = []
        if flags & 1:
            what.append("bit 0: the fused clip + update launch applied a clip factor from stale "
                        "partials (rerun with BA3C_FUSED_UPDATE=0)")
        if flags & 2:
            what.append("bit 1: a one-launch bucket clip (ba3c_clip_grads_range) gave up waiting, "
                        "so invalid clipped gradients entered the all-reduce")
        if flags & 4:
            what.append("bit 2: a chained launch's waiting workgroups gave up waiting for their "
                        "producers (rerun with BA3C_CHAIN=0)")
        if flags & ~7:
            what.append("unknown bits 0x%x" % (flags & ~7))
        return "; ".join(what)

    def check_device_errors(self):
        """Abort on an in-launch wait that gave up (ba3c_device_errors != 0): the parameters
        are then no longer the reference's.  Called where the host already synchronises
        (run_step, the metrics flush of train.py, bench.py after the timed steps); it
        synchronises the device itself."""
        f = self.engine.device_errors() if hasattr(self.engine, "device_errors") else 0
        if f:
            raise RuntimeError("device error flags 0x%x after global step %d: %s"
                               % (f, self.global_step, self.describe_device_errors(f)))

    def train_step(self, state, action, futurereward):
        """Device-side step (used by bench.py).  No host synchronisation, except with backup
        workers (SyncReplicasOptimizer with replicas_to_aggregate < world): each step then
        synchronises the stream and all-gathers the ranks' ready times on the host before a
        flat (not bucketed) all-reduce, so its step times are not comparable with k = N."""
        opt = self.optimizer
        # backup workers pick the first k ranks once the whole gradient is ready: flat path
        if (isinstance(opt, SyncReplicasOptimizer) and self._fused_clip and opt.bucketed
                and not opt.backup_workers):
            self._bucketed_sync_step(state, action, futurereward)
            self.global_step += 1
            return
        if self._defer_reduce and self._fused_clip and not isinstance(opt, SyncReplicasOptimizer):
            self.model.train_phase = 3
        try:
            self.model.build_graph([state, action, futurereward])
        finally:
            self.model.train_phase = 0
        if isinstance(opt, SyncReplicasOptimizer):
            if self._fused_clip:
                opt.aggregate(self.engine)
            else:
                self.process_grads()
                opt.allreduce(self.engine)
            opt.apply_gradients(self.engine)
        elif self._fused_clip:
            opt.apply_gradients(self.engine, fuse_clip=True)
        else:
            self.process_grads()
            opt.apply_gradients(self.engine)
        self.global_step += 1

    def _bucketed_sync_step(self, state, action, futurereward):
        """Data-parallel step with the gradient exchange in two buckets: phase 1 of the pass
        (forward, loss, heads + fc1 backward) -> clip + async RCCL sum of the fc1 + heads
        bucket -> phase 2 (conv backward, overlapping that all-reduce) -> clip + RCCL sum of
        the conv bucket -> wait -> the identical update on every rank (grad_scale = 1/N).
        With a `timeline` attached (ExchangeTimeline, bench.py) the step records HIP events
        at each of these points."""
        eng, opt, m = self.engine, self.optimizer, self.model
        tb, off = eng.bucket_split()
        nt, total = len(eng.layout), eng.grads.numel()
        inputs = [state, action, futurereward]
        tl = self.timeline.new_step() if self.timeline is not None else None
        mark = (lambda k: tl[k].record()) if tl is not None else (lambda k: None)
        if self._mid is None and eng.grads.is_cuda:
            # recorded by every phase-2 pass after conv3's launches (ba3c_set_phase2_event)
            self._mid = hipevent.HipEvent(hipevent.HIP_EVENT_DISABLE_TIMING
                                          | hipevent.HIP_EVENT_RELEASE_TO_DEVICE)
            eng.set_phase2_event(self._mid)
        held = self._xchg_held
        mark("start")
        try:
            # phase 1; BA3C_XCHG_HELD=1: phase 4, its fc1 + heads reduction held back for the
            # exchange stream
            m.train_phase = 4 if held else 1
            m.build_graph(inputs)
            mark("phase1_end")
            if not held:
                eng.clip_grads_range(tb, nt)     # the bucket's clip (one launch)
            m.train_phase = 2
            m.build_graph(inputs)
        finally:
            m.train_phase = 0
        # the fc1 + heads bucket's sum on the exchange stream from the phase-2 event on, beside
        # conv2..conv0's backward (held: its reduction and clip first)
        work = opt.aggregate_held_bucket_async(
            eng, self._mid, tb, nt, off, total, held=held,
            marks=tl and (tl["fc1_start"], tl["fc1_ready"], tl["fc1_ar_begin"], tl["fc1_ar_end"]))
        work2 = opt.aggregate_bucket_async(
            eng, 0, tb, 0, off, last=True,
            marks=tl and (tl["conv_ready"], tl["conv_ar_begin"], tl["conv_ar_end"]))
        for w in (work, work2):
            if w is not None:
                w.wait()
        mark("exchanged")
        opt.apply_gradients(eng)
        mark("end")

    timeline = None
    _mid = None

    def capture_step(self, state, action, futurereward, warmup=2):
        """Capture one full step (fwd+bwd+clip+update) on static input tensors as a hipGraph
        (torch.cuda.CUDAGraph over the HIP stream).  Returns a callable that replays it; the
        caller refills `state`/`action`/`futurereward` in place between replays.  Adam's
        beta powers move to the device so every replay uses the right bias correction.
        The `warmup` eager steps that precede the capture (allocator / library warm-up) are
        undone: parameters, optimizer slots and beta powers are restored afterwards, so
        capturing does not train the model."""
        opt = self.optimizer
        if isinstance(opt, SyncReplicasOptimizer) and opt.backup_workers:
            raise ValueError("backup workers choose the aggregated ranks on the host each "
                             "step; such a step cannot be captured as a graph")
        inner = opt._opt if isinstance(opt, SyncReplicasOptimizer) else opt
        if hasattr(inner, "use_device_state"):
            inner.use_device_state(self.engine.device)
        if inner.slots is None:
            inner.slots = inner._init_slots(self.engine)
        saved = [t.clone() for t in [self.engine.params] + list(inner.slots)
                 + ([inner.dev_powers] if inner.dev_powers is not None else [])]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.train_step(state, action, futurereward)
            live = [self.engine.params] + list(inner.slots) + (
                [inner.dev_powers] if inner.dev_powers is not None else [])
            for dst, src in zip(live, saved):
                dst.copy_(src)
        torch.cuda.current_stream().wait_stream(side)
        self.global_step -= warmup
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            self.train_step(state, action, futurereward)
        self.global_step -= 1                 # capture records the step, it does not run it

        def replay():
            graph.replay()
            self.global_step += 1
        return replay

    def run_step(self, batch):
        """batch = [state, action, futurereward, ts, init_R, isOver] (train.py:432) as numpy or
        tensors; returns the TfDictOp dict incl. global_step and dp_per_s (multigpu.py:307-313)."""
        t0 = time.time()
        dev = self.engine.device
        state = torch.as_tensor(np.asarray(batch[0], dtype=np.uint8)).to(dev)
        action = torch.as_tensor(np.asarray(batch[1], dtype=np.int64)).to(dev)
        R = torch.as_tensor(np.asarray(batch[2], dtype=np.float32)).to(dev)
        self.train_step(state, action, R)
        out = self.model.scalars_dict()      # synchronises the stream
        self.check_device_errors()
        if len(batch) > 3 and batch[3] is not None:
            out["delay"] = float(np.mean(self.global_step - np.asarray(batch[3], np.float64)))
        out["global_step"] = self.global_step
        self.step_ms.append((time.time() - t0) * 1000.0)
        out["dp_per_s"] = 1000.0 / np.mean(self.step_ms[-20:]) * state.shape[0]
        return out
