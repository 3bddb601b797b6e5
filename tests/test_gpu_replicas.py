"""Two real HIP replicas exchanging gradients (BASELINE configs[3] path, train.py:598-606,
train/multigpu.py:157,194) on the one GPU of the test box.

Two processes, each with its own Ba3cEngine on cuda:0, run Ba3cTrainer with
SyncReplicasOptimizer over a world-size-2 gloo group (RCCL refuses two ranks on one device, so
the exchange is host-staged: SyncReplicasOptimizer._staged).  Everything else is the product
path of the N-GPU run: the phase-split backward (ba3c_train_grads_phase), the per-replica
clip of each bucket (ba3c_clip_grads_range), the asynchronous bucket all-reduce beside the
conv backward (trainer.py _bucketed_sync_step), the grad_scale = 1/N update, and rank 0's
variables broadcast at start.  Checked: the replicas stay bit-identical, equal a one-process
emulation (sum of the two clipped buffers, one apply) bit for bit, and the oracle's
SyncReplicas step within the north-star tolerance.  The backup-worker case (num_grad=1 of 2,
train.py:601-602) runs the same replicas with a fixed arrival order: each step only the first
replica's clipped gradients enter the exchange and the update is bit-identical to applying
that replica's buffer alone.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import ba3c_oracle as O
from test_gpu_parity import GRAD_TOL, as64, rel

pytestmark = pytest.mark.gpu

B, F, S, A = 16, 128, 4, 4
CFG = {"fc_neurons": F, "fc_splits": S}


def _batch(step, rank):
    rs = np.random.RandomState(700 + 10 * step + rank)
    return (rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8),
            rs.randint(0, A, size=B).astype(np.int64), rs.normal(size=B).astype(np.float32))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# backup-worker case: the rank whose gradients arrive first at each step
FIRST = [1, 0]


def _arrival(rank, step):
    return 0.0 if rank == FIRST[step] else 1.0


def _worker(rank, world, port, bucketed, out, k=None):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "distributed-ba3c_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ba3c_amd.model import Model
        from ba3c_amd.optimizer import AdamOptimizer, SyncReplicasOptimizer
        from ba3c_amd.trainer import Ba3cTrainer, TrainConfig
        # different initial variables per rank: the trainer broadcasts rank 0's
        m = Model(num_actions=A, fc_neurons=F, fc_splits=S, batch_size=B, max_batch=B, seed=20 + rank)
        own = m.engine.params.cpu().numpy()
        opt = SyncReplicasOptimizer(AdamOptimizer(1e-3, 0.8, 0.75, 1e-8), k or world, world,
                                    arrival_fn=_arrival if k else None)
        opt.bucketed = bucketed
        tr = Ba3cTrainer(TrainConfig(model=m, optimizer=opt))
        p0 = m.engine.params.cpu().numpy()
        ps = []
        for step in range(2):
            s, a, r = (torch.from_numpy(x).cuda() for x in _batch(step, rank))
            tr.train_step(s, a, r)
            ps.append(m.engine.params.cpu().numpy())
        tr.check_device_errors()
        out[rank] = (own, p0, ps)
    finally:
        dist.destroy_process_group()


def _emulate(p0_flat, only_first=False):
    """One process, one engine: per replica train_grads + clip_grads, the sum, one
    apply_update(grad_scale=1/2, fuse_clip=0) — what the exchange must amount to (backup
    workers: the first replica's buffer alone, grad_scale=1)."""
    from ba3c_amd.engine import Ba3cEngine
    from ba3c_amd.optimizer import AdamOptimizer
    eng = Ba3cEngine(num_actions=A, fc_neurons=F, fc_splits=S, max_batch=B)
    eng.params.copy_(torch.from_numpy(p0_flat))
    opt = AdamOptimizer(1e-3, 0.8, 0.75, 1e-8)
    ps = []
    for step in range(2):
        total = torch.zeros_like(eng.grads)
        for rank in ([FIRST[step]] if only_first else range(2)):
            s, a, r = (torch.from_numpy(x).cuda() for x in _batch(step, rank))
            eng.train_grads(s, a, r)
            eng.clip_grads()
            total += eng.grads
        eng.grads.copy_(total)
        opt.apply_gradients(eng, grad_scale=1.0 if only_first else 0.5, fuse_clip=False)
        ps.append(eng.params.cpu().numpy())
    return eng, ps


@pytest.mark.parametrize("bucketed", [True, False])
def test_two_hip_replicas_exchange_gradients(bucketed):
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), bucketed, out), nprocs=world, join=True,
                       start_method="spawn")
    (own_a, p0a, pa), (own_b, p0b, pb) = out[0], out[1]
    assert not np.array_equal(own_a, own_b)             # they were initialised apart ...
    np.testing.assert_array_equal(p0a, own_a)           # ... rank 0's variables were broadcast
    np.testing.assert_array_equal(p0b, own_a)
    for step in range(2):                               # and they are one model after each step
        np.testing.assert_array_equal(pa[step], pb[step])
    eng, emu = _emulate(p0a)
    for step in range(2):
        np.testing.assert_array_equal(pa[step], emu[step])
    # the oracle's SyncReplicas step from the same variables: mean of the per-replica clipped
    # gradients, one TF Adam apply (each later step is the same arithmetic: the emulation's
    # steps are held to the oracle step by step in test_gpu_bench_path.py)
    params = as64({n: p0a[o:o + k].reshape(sh) for n, o, k, sh in eng.layout})
    slots = O.init_slots(params, "adam", 0.8, 0.75)
    newp, _, _, g = O.train_step(params, slots, 1,
                                 [(x[0], x[1], x[2].astype(np.float64))
                                  for x in (_batch(0, 0), _batch(0, 1))],
                                 CFG, lr=1e-3, beta1=0.8, beta2=0.75, eps=1e-8)
    got = {n: pa[0][o:o + k].reshape(sh) for n, o, k, sh in eng.layout}
    for k in g:
        d_got = got[k].astype(np.float64) - params[k]
        d_ref = newp[k] - params[k]
        mask = np.abs(g[k]) > 1e-4 * max(np.abs(g[k]).max(), 1e-30)
        if mask.any():
            assert rel(d_got[mask], d_ref[mask]) < GRAD_TOL, k


def test_two_hip_replicas_backup_worker_drops_the_late_gradients():
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), True, out, 1), nprocs=world, join=True,
                       start_method="spawn")
    (_, p0a, pa), (_, _, pb) = out[0], out[1]
    _, emu = _emulate(p0a, only_first=True)
    _, both = _emulate(p0a)
    for step in range(2):
        np.testing.assert_array_equal(pa[step], pb[step])
        np.testing.assert_array_equal(pa[step], emu[step])
    assert not np.array_equal(pa[0], both[0])           # the dropped replica's gradients mattered
