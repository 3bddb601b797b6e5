"""TF-1.2 optimizers over the flat buffers (train.py:582-606) and SyncReplicasOptimizer.

Slot initial values, the float32 beta-power variables and the scalar arithmetic follow the
TF-1.2 CPU functors.  Every apply is ONE fused HIP kernel over
the flat parameter buffer (`ba3c_apply_update`), optionally with clip_by_average_norm fused
in (single replica).  SyncReplicasOptimizer replaces the parameter-server accumulators with
an RCCL all-reduce of the flat clipped-gradient buffer (torch.distributed 'nccl' == RCCL).
"""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from . import hipevent

_f = np.float32


class Optimizer(object):
    opt_id = None
    n_slots = 0

    def __init__(self, learning_rate):
        self.learning_rate = float(learning_rate)   # non-trainable 'learning_rate' var (train.py:536)
        self.slots = None

    def _init_slots(self, engine):
        raise NotImplementedError

    def _hparams(self):
        return dict(lr=self.learning_rate, beta1=0.0, beta2=0.0, epsilon=0.0, beta1_power=0.5,
                    beta2_power=0.5, decay=0.0, momentum=0.0, rho=0.0)

    def _after_apply(self):
        pass

    dev_powers = None

    def apply_gradients(self, engine, grad_scale=1.0, fuse_clip=False, grads=None):
        """optimizer.apply_gradients(grads) (train/multigpu.py:194) over engine.grads."""
        if self.slots is None:
            self.slots = self._init_slots(engine)
        s0 = self.slots[0] if len(self.slots) > 0 else None
        s1 = self.slots[1] if len(self.slots) > 1 else None
        engine.apply_update(self.opt_id, s0, s1, self._hparams(), grad_scale=grad_scale,
                            fuse_clip=fuse_clip, grads=grads, dev_powers=self.dev_powers)
        self._after_apply()

    def slot_dict(self, engine, i):
        return engine.state_dict(self.slots[i])


class AdamOptimizer(Optimizer):
    """tf.train.AdamOptimizer(lr, beta1, beta2, epsilon) — m, v zero-initialised; beta powers
    are float32 variables initialised to beta1/beta2 and multiplied after each apply."""
    opt_id = "adam"

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8):
        super(AdamOptimizer, self).__init__(learning_rate)
        self.beta1, self.beta2, self.epsilon = float(beta1), float(beta2), float(epsilon)
        self.beta1_power = _f(beta1)
        self.beta2_power = _f(beta2)

    def _init_slots(self, engine):
        return [engine.zeros_like_flat(), engine.zeros_like_flat()]

    def _hparams(self):
        h = super(AdamOptimizer, self)._hparams()
        h.update(beta1=self.beta1, beta2=self.beta2, epsilon=self.epsilon,
                 beta1_power=float(self.beta1_power), beta2_power=float(self.beta2_power))
        return h

    def _after_apply(self):
        if self.dev_powers is not None:
            return                       # the GPU multiplies its own copy (graph-safe)
        self.beta1_power = _f(self.beta1_power * _f(self.beta1))
        self.beta2_power = _f(self.beta2_power * _f(self.beta2))

    def use_device_state(self, device):
        """Move beta1_power/beta2_power to a device tensor updated by the update kernel's
        stream, so the whole step can be captured once and replayed as a hipGraph."""
        if self.dev_powers is None:
            self.dev_powers = torch.tensor([self.beta1_power, self.beta2_power],
                                           dtype=torch.float32, device=device)

    def powers(self):
        if self.dev_powers is not None:
            v = self.dev_powers.cpu().numpy()
            return _f(v[0]), _f(v[1])
        return self.beta1_power, self.beta2_power


class RMSPropOptimizer(Optimizer):
    """tf.train.RMSPropOptimizer(lr) with TF-1.2 defaults; 'rms' slot initialised to ONES."""
    opt_id = "rms"

    def __init__(self, learning_rate, decay=0.9, momentum=0.0, epsilon=1e-10):
        super(RMSPropOptimizer, self).__init__(learning_rate)
        self.decay, self.momentum, self.epsilon = float(decay), float(momentum), float(epsilon)

    def _init_slots(self, engine):
        return [engine.zeros_like_flat(1.0), engine.zeros_like_flat()]

    def _hparams(self):
        h = super(RMSPropOptimizer, self)._hparams()
        h.update(decay=self.decay, momentum=self.momentum, epsilon=self.epsilon)
        return h


class GradientDescentOptimizer(Optimizer):
    opt_id = "gd"

    def _init_slots(self, engine):
        return []


class MomentumOptimizer(Optimizer):
    opt_id = "momentum"

    def __init__(self, learning_rate, momentum=0.9):
        super(MomentumOptimizer, self).__init__(learning_rate)
        self.momentum = float(momentum)

    def _init_slots(self, engine):
        return [engine.zeros_like_flat()]

    def _hparams(self):
        h = super(MomentumOptimizer, self)._hparams()
        h.update(momentum=self.momentum)
        return h


class AdagradOptimizer(Optimizer):
    opt_id = "adagrad"

    def __init__(self, learning_rate, initial_accumulator_value=0.1):
        super(AdagradOptimizer, self).__init__(learning_rate)
        self.init_acc = float(initial_accumulator_value)

    def _init_slots(self, engine):
        return [engine.zeros_like_flat(self.init_acc)]


class AdadeltaOptimizer(Optimizer):
    opt_id = "adadelta"

    def __init__(self, learning_rate=0.001, rho=0.95, epsilon=1e-8):
        super(AdadeltaOptimizer, self).__init__(learning_rate)
        self.rho, self.epsilon = float(rho), float(epsilon)

    def _init_slots(self, engine):
        return [engine.zeros_like_flat(), engine.zeros_like_flat()]

    def _hparams(self):
        h = super(AdadeltaOptimizer, self)._hparams()
        h.update(rho=self.rho, epsilon=self.epsilon)
        return h


def make_optimizer(name, lr, beta1=0.9, beta2=0.999, epsilon=1e-8):
    """The `-o` switch of run_job.py / get_config (train.py:583-597)."""
    if name == "adam":
        return AdamOptimizer(lr, beta1=beta1, beta2=beta2, epsilon=epsilon)
    if name == "gd":
        return GradientDescentOptimizer(lr)
    if name == "adagrad":
        return AdagradOptimizer(lr)
    if name == "adadelta":
        return AdadeltaOptimizer(lr, epsilon=1e-3)
    if name == "momentum":
        return MomentumOptimizer(lr, momentum=0.9)
    if name == "rms":
        return RMSPropOptimizer(lr)
    raise ValueError("unknown optimizer %r" % name)


class _StagedWork(object):
    """Work handle of a host-staged all-reduce: wait() completes it and copies the sum back
    into the device buffer (on `stream`, default the current one, so later kernels see it);
    `end` (a timing event) is recorded on that stream after the copy."""

    def __init__(self, work, host, dst, stream=None, end=None):
        self.work, self.host, self.dst = work, host, dst
        self.stream, self.end = stream, end

    def wait(self):
        self.work.wait()
        if self.stream is None:
            self.dst.copy_(self.host)
            return True
        with torch.cuda.stream(self.stream):
            self.dst.copy_(self.host)
            if self.end is not None:
                self.end.record(self.stream)
        hipevent.wait_stream(torch.cuda.current_stream(self.dst.device), self.stream)
        return True


class _StreamJoin(object):
    """Work handle of an all-reduce issued on the exchange stream: wait() makes the current
    stream wait for it (no host synchronisation)."""

    def __init__(self, stream):
        self.stream = stream
        self.joined = False      # set once the current stream already waits for the sum

    def wait(self):
        if not self.joined:
            hipevent.wait_stream(torch.cuda.current_stream(self.stream.device), self.stream)
            self.joined = True
        return True


class SyncReplicasOptimizer(object):
    """tf.train.SyncReplicasOptimizer(opt, replicas_to_aggregate, total_num_replicas)
    (train.py:598-606) on one node: every rank clips its own gradients, the flat buffer is
    summed over RCCL (one all-reduce of 1.3-3.8 MB), and every rank applies the same update
    with grad_scale = 1/N, so replicas stay bit-identical.

    Backup workers (`replicas_to_aggregate` k < `total_num_replicas` N, the reference's
    `--num_grad` below the worker count, train.py:601-602): TF's accumulator averages the
    first k gradients that arrive for the current global step and drops the late ones as
    stale (their local_step is behind once the chief has applied).  Here each step's arrival
    order is the order in which the ranks' clipped gradients became ready on the device
    (host CLOCK_MONOTONIC after a stream synchronise, shared by every process on the node,
    exchanged with one all-gather of N doubles); the first k (ties: lower rank) contribute,
    the others contribute zeros to the same all-reduce, and every rank applies the mean over
    exactly k (grad_scale = 1/k).  All ranks then continue from the new parameters, as a
    late TF worker does after dequeuing its next token.  Differences, documented: the
    collective still waits for the stragglers (a synchronous all-reduce has no early exit,
    so backup workers change the arithmetic, not the step time), and the mean is over
    exactly k where TF's take_grad may average more that arrived before it ran."""

    def __init__(self, opt, replicas_to_aggregate=None, total_num_replicas=None, group=None,
                 arrival_fn=None):
        self._opt = opt
        self.group = group
        self.distributed = dist.is_available() and dist.is_initialized()
        world = dist.get_world_size(group) if self.distributed else 1
        self.total_num_replicas = total_num_replicas or world
        self.replicas_to_aggregate = replicas_to_aggregate or self.total_num_replicas
        if self.total_num_replicas != world:
            raise ValueError("every rank of the group is one replica: total_num_replicas must "
                             "be world_size=%d (got %s)" % (world, total_num_replicas))
        if not 1 <= self.replicas_to_aggregate <= world:
            raise ValueError("replicas_to_aggregate must be in [1, %d] (got %s)"
                             % (world, replicas_to_aggregate))
        self.world = world
        self.rank = dist.get_rank(group) if self.distributed else 0
        # arrival_fn(rank, step) -> float: a fixed arrival order for tests; None measures it
        self.arrival_fn = arrival_fn
        # measured arrivals compare CLOCK_MONOTONIC readings, which only one node shares
        lws = os.environ.get("LOCAL_WORLD_SIZE")
        if (world - self.replicas_to_aggregate) and arrival_fn is None and lws is not None \
                and int(lws) != world:
            raise ValueError("backup workers order arrivals by the node's monotonic clock: the "
                             "group must be one node (LOCAL_WORLD_SIZE=%s, world size %d)"
                             % (lws, world))
        self.local_step = 0
        self.last_aggregated = list(range(world))
        self.dropped = 0                      # this rank's gradients dropped as stale

    @property
    def backup_workers(self):
        return self.world - self.replicas_to_aggregate

    @property
    def learning_rate(self):
        return self._opt.learning_rate

    @learning_rate.setter
    def learning_rate(self, v):
        self._opt.learning_rate = v

    @property
    def slots(self):
        return self._opt.slots

    def powers(self):
        return self._opt.powers()

    def broadcast_variables(self, engine, src=0):
        """Every replica starts from rank `src`'s variables (and optimizer slots, e.g. after a
        restore), as all workers of the reference read the one PS copy (train.py:512-515)."""
        if not self.distributed:
            return
        for t in [engine.params] + list(self._opt.slots or []) + (
                [self._opt.dev_powers] if self._opt.dev_powers is not None else []):
            if self._staged(t):
                host = t.cpu()
                dist.broadcast(host, src=src, group=self.group)
                t.copy_(host)
            else:
                dist.broadcast(t, src=src, group=self.group)

    def _staged(self, t):
        """gloo group + device tensor (several replicas sharing one GPU, where RCCL refuses
        two ranks on one device; tests and CPU rehearsals): the exchange goes through a host
        copy.  RCCL ('nccl') takes the device buffer directly."""
        return t.is_cuda and dist.get_backend(self.group) == "gloo"

    def _all_reduce(self, t, async_op=False):
        if not self._staged(t):
            return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
        host = t.cpu()                     # waits for the producing kernels on this stream
        work = dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        staged = _StagedWork(work, host, t)
        if async_op:
            return staged
        staged.wait()
        return None

    def allreduce(self, engine):
        """Sum of the replicas' flat gradient buffers over RCCL ('nccl' backend), issued on the
        current HIP stream; runs whenever a process group exists (also at world size 1).  With
        backup workers only the first k ranks' buffers enter the sum (select_first)."""
        if self.distributed and self.backup_workers:
            self.last_aggregated = self.select_first(engine)
            if self.rank not in self.last_aggregated:
                engine.grads.zero_()          # stale: dropped, as TF's accumulator does
                self.dropped += 1
        self.local_step += 1
        if self.distributed:
            self._all_reduce(engine.grads)

    def aggregate(self, engine):
        """Per-replica clip (multigpu.py:157) then the RCCL sum of the clipped buffer."""
        engine.clip_grads()
        self.allreduce(engine)

    def _arrival(self, engine):
        if self.arrival_fn is not None:
            return float(self.arrival_fn(self.rank, self.local_step))
        if engine.grads.is_cuda:
            torch.cuda.current_stream(engine.grads.device).synchronize()
        return time.monotonic()

    def select_first(self, engine):
        """Ranks whose gradients this step aggregates: the first k to arrive (one all-gather
        of every rank's arrival time; ties go to the lower rank).  Returns the sorted list."""
        t = torch.tensor([self._arrival(engine)], dtype=torch.float64)
        if dist.get_backend(self.group) != "gloo":
            t = t.to(engine.grads.device)
        times = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(times, t, group=self.group)
        order = sorted(range(self.world), key=lambda r: (float(times[r][0]), r))
        return sorted(order[:self.replicas_to_aggregate])

    # bucketed exchange: the fc1 + heads tensors (~90 % of the parameters at
    # F=512) are final after the first half of the backward pass, so their clip and RCCL sum
    # run beside the conv layers' backward; the conv bucket follows at the end of the pass
    bucketed = True
    _comm = None

    def comm_stream(self, device):
        """The exchange stream of the bucketed step: each bucket's sum is issued on it after
        the bucket's clip, so its start and end can be marked with HIP events in the same
        stream order as the collective (torch's NCCL stream joins it on wait()).

        High priority by default (BA3C_XCHG_PRIORITY=0: normal): the backward's persistent conv
        kernels fill every CU, so the collective's workgroups can only start at a kernel
        boundary, and there the dispatcher should place them ahead of the next conv kernel's
        workgroups rather than after all of them."""
        if self._comm is None:
            flag = os.environ.get("BA3C_XCHG_PRIORITY", "1")
            if flag not in ("0", "1"):
                raise ValueError("BA3C_XCHG_PRIORITY must be 0 or 1 (got %r)" % flag)
            self._comm = torch.cuda.Stream(device=device, priority=-1 if flag == "1" else 0)
        return self._comm

    # RCCL driven directly (rccl.py) for the bucket sums on a 'nccl' group; BA3C_DIRECT_RCCL=0
    # keeps torch's collective (its own stream, joined with events)
    _rccl = None

    def direct_rccl(self, device):
        """The direct RCCL communicator of this group (created on first use, collectively), or
        None on a gloo group or with BA3C_DIRECT_RCCL=0.

        Every rank takes the same path: the library load, the communicator and an
        exact-sum self-test through it are each agreed on with a MIN all-reduce over the
        process group, so one rank falling back to torch's collective while the others wait on
        the direct communicator cannot happen."""
        flag = os.environ.get("BA3C_DIRECT_RCCL", "1")
        if flag not in ("0", "1"):
            raise ValueError("BA3C_DIRECT_RCCL must be 0 or 1 (got %r)" % flag)
        if flag == "0" or dist.get_backend(self.group) != "nccl" or self._rccl is False:
            return None
        if self._rccl is None:
            from . import rccl as R

            def agree(ok, what):
                t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
                if int(t.item()) == 0:
                    print("ba3c: direct RCCL unavailable on some rank (%s); every rank uses "
                          "torch's collective" % what, file=sys.stderr)
                    return False
                return True
            err = None
            try:
                R._lib()
            except (OSError, AttributeError) as e:
                err = e
            if not agree(err is None, "library: %s" % err):
                self._rccl = False
                return None
            comm = None
            try:
                comm = R.RcclComm(self.group, device)
                ok = comm.selftest()
                err = None if ok else "exact-sum self-test mismatch"
            except R.RcclError as e:
                err = e
            if not agree(err is None, "communicator: %s" % err):
                if comm is not None:
                    comm.close()
                self._rccl = False
                return None
            self._rccl = comm
            import atexit
            atexit.register(self._close_at_exit)
        return self._rccl

    def rccl_info(self):
        """RcclComm.info() of the direct communicator, or None when torch's collective runs."""
        return self._rccl.info() if self._rccl else None

    def close(self):
        """Destroy the direct RCCL communicator (before dist.destroy_process_group), so no
        RCCL proxy thread outlives the process group.  Waits for the device first: call it
        only when every rank reached the same point (bench.py does, after a barrier)."""
        if self._rccl:
            torch.cuda.synchronize(self._rccl.device)
            self._rccl.close()
            self._rccl = None

    def _close_at_exit(self):
        """Interpreter exit without an explicit close() (train.py, torchrun, a rank leaving on
        an exception): abort the communicator instead of synchronising, since an all-reduce
        still waiting on a dead or diverged peer would never finish and the rank would hang
        at exit instead of failing."""
        if self._rccl:
            self._rccl.close(abort=True)
            self._rccl = None

    # HIP event recorded on the exchange stream after the last asynchronous bucket sum of the
    # step; the next sum on the same communicator from another stream waits for it, so the
    # order of two collectives on one communicator never rests on RCCL's cross-stream
    # serialisation
    _ar_done = None
    _ar_event = None
    _ready_event = None
    _fc1_join = None

    def aggregate_held_bucket_async(self, engine, mid, t0, t1, off0, off1, marks=None, held=True):
        """The N>1 step's first bucket (fc1 + heads): on the exchange stream, once `mid`
        (recorded in phase 2 right after conv3's launches) has passed, the bucket's sum.
        Starting there puts the collective's workgroups at the boundary before conv2's launch,
        whose short non-persistent workgroups the dispatcher rebalances, rather than beside
        conv3's persistent ones.  `held` (a phase-4 pass, BA3C_XCHG_HELD=1): the held reduction
        of the bucket's weight gradients and the bucket's clip in its two-launch form (it runs
        beside phase 2's kernels, so its workgroups cannot assume co-residency) run there
        first; otherwise the caller clipped the bucket on its own stream after phase 1.
        `marks`: (start, ready, begin, end) timing events on the exchange stream.  Returns the
        work handle (always: the update must join the exchange stream)."""
        start, ready, begin, end = marks if marks is not None else (None, None, None, None)
        dev = engine.grads.device
        buf = engine.grads[off0:off1]
        if not buf.is_cuda:                   # CPU engines (tests): no streams
            if held:
                engine.launch_held()
                engine.clip_grads_range(t0, t1)
            return self._all_reduce(buf, async_op=True) if self.distributed else None
        rccl = self.direct_rccl(dev) if self.distributed else None   # (collective on first use)
        comm = self.comm_stream(dev)
        if isinstance(mid, hipevent.HipEvent):
            mid.wait(comm)
        else:
            comm.wait_event(mid)
        join = _StreamJoin(comm)
        with torch.cuda.stream(comm):
            if start is not None:
                start.record(comm)
            if held:
                engine.launch_held(comm)
                engine.clip_grads_range(t0, t1, no_residency=True)
            if ready is not None:
                ready.record(comm)
            if not self.distributed:
                return join
            if begin is not None:
                begin.record(comm)
            if self._staged(buf):
                host = buf.cpu()              # host-staged (gloo): waits for the clip
                work = dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                return _StagedWork(work, host, buf, stream=comm, end=end)
            if rccl is not None:
                rccl.all_reduce_sum(buf, comm)
                self._occupy(engine, comm)
                if self._ar_event is None:
                    self._ar_event = hipevent.join_event()
                self._ar_event.record(comm)
                self._ar_done = self._ar_event
                self._fc1_join = join
            else:
                work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                work.wait()                   # `comm` waits for the collective's stream
                self._occupy(engine, comm)
            if end is not None:
                end.record(comm)
        return join

    def aggregate_bucket_async(self, engine, t0, t1, off0, off1, marks=None, last=False):
        """Clip tensors [t0, t1) and start the RCCL sum of flat range [off0, off1); returns
        the work handle (None when there is nothing to join).  The sum runs on the exchange
        stream, except the `last` bucket's on a direct-RCCL group: the update waits for it
        next, so it is enqueued on the current stream itself.  `marks`: (ready, begin, end)
        timing events — `ready` on the current stream after the clip, begin / end around the
        sum on the stream that runs it."""
        engine.clip_grads_range(t0, t1)
        ready, begin, end = marks if marks is not None else (None, None, None)
        cur = torch.cuda.current_stream(engine.grads.device) if engine.grads.is_cuda else None
        if ready is not None:
            ready.record(cur)
        if not self.distributed:
            return None
        buf = engine.grads[off0:off1]
        if not buf.is_cuda:
            return self._all_reduce(buf, async_op=True)
        rccl = self.direct_rccl(buf.device)
        if rccl is not None and last:
            if self._ar_done is not None:
                # the exchange stream's sum is enqueued first; this wait also joins it, so the
                # update needs no second cross-stream wait
                if isinstance(self._ar_done, hipevent.HipEvent):
                    self._ar_done.wait(cur)
                else:
                    cur.wait_event(self._ar_done)
                self._ar_done = None
                if self._fc1_join is not None:
                    self._fc1_join.joined = True
                    self._fc1_join = None
            if begin is not None:
                begin.record(cur)
            rccl.all_reduce_sum(buf, cur)
            if end is not None:
                end.record(cur)
            return None
        comm = self.comm_stream(buf.device)
        if self._ready_event is None:
            self._ready_event = hipevent.join_event()
        hipevent.wait_stream(comm, cur, self._ready_event)
        with torch.cuda.stream(comm):
            if begin is not None:
                begin.record(comm)
            if self._staged(buf):
                host = buf.cpu()              # host-staged (gloo): waits for the clip
                work = dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                return _StagedWork(work, host, buf, stream=comm, end=end)
            if rccl is not None:
                rccl.all_reduce_sum(buf, comm)
                self._occupy(engine, comm)
                if self._ar_event is None:
                    self._ar_event = hipevent.join_event()
                self._ar_event.record(comm)
                self._ar_done = self._ar_event
            else:
                work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                work.wait()                   # `comm` waits for the collective's stream
                self._occupy(engine, comm)
            if end is not None:
                end.record(comm)
        join = _StreamJoin(comm)
        if rccl is not None:
            self._fc1_join = join
        return join

    # bench.py --occupy: (K, microseconds) — after the fc1 + heads bucket's sum, a launch on the
    # exchange stream holds K CUs for that long (ba3c_occupy_cus), standing in for the CUs
    # RCCL's channel workgroups take on a multi-GPU node while phase 2 runs.  None: off.
    occupy = None

    def _occupy(self, engine, stream):
        if self.occupy:
            engine.occupy_cus(stream, *self.occupy)

    def apply_gradients(self, engine):
        self._opt.apply_gradients(engine, grad_scale=1.0 / self.replicas_to_aggregate,
                                  fuse_clip=False)
