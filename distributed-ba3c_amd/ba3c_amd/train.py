"""`python -m ba3c_amd.train` — the single-node launcher on the reference's flag surface.

Replaces run_job.py:13-148 -> distributed_tensorpack_mkl.sh -> OpenAIGym/train.py:649-724
(get_config :505-638): from the same flags it builds the Model (train.py:517), the optimizer
(`-o`, :582-597), SyncReplicasOptimizer for `--use_sync -g N` (:598-606, here an RCCL
all-reduce over the node's GPUs), the trainer and the actor-learner loop (simulator master +
predictor + BatchData, :520-534 — with the synthetic on-device environment, gym/ALE being
absent), plus the DebugLogCallback metrics channels and PeriodicPerStepCallback(ModelSaver)
(:608-630) and `--load` (SaverRestore, :706-707).

One process per GPU: launch N > 1 with
    torchrun --nproc-per-node N --master-addr 127.0.0.1 -m ba3c_amd.train --use_sync -g N ...
The process group ('nccl' = RCCL) is created before any other GPU work.  Each rank seeds its
numpy stream with its worker index (train.py:678-679); variables start identical on every
rank (rank 0's are broadcast).
"""
import json
import os
import socket
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

from .flags import build_parser, resolve


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def model_config(args):
    """The Model / engine geometry the flags select (train.py:95, :216-243)."""
    return dict(num_actions=args.num_actions, channels=args.channels, fc_neurons=args.fc_neurons,
                fc_splits=args.fc_splits, replace_with_conv=bool(args.replace_with_conv),
                ps=args.ps, batch_size=args.batch_size)


def optimizer_config(args):
    """`-o` and its hyper-parameters (train.py:582-597)."""
    return dict(name=args.optimizer, lr=args.lr, beta1=args.beta1, beta2=args.beta2,
                epsilon=args.epsilon)


def check_distributed(args, world):
    """Synchronous data parallelism only (the asynchronous PS mode has no all-reduce
    equivalent): --use_sync with 1 <= --ngrads <= world size.  --ngrads below the world size
    keeps the reference's backup workers (train.py:601-602): each step averages the first
    `ngrads` ranks' gradients and drops the rest as stale (SyncReplicasOptimizer)."""
    if world > 1 and not args.use_sync:
        raise SystemExit("world size %d: multi-GPU training is synchronous (RCCL all-reduce); "
                         "pass --use_sync -g %d" % (world, world))
    if args.use_sync and not 1 <= args.ngrads <= world:
        raise SystemExit("--ngrads %d must be in [1, %d] (the number of GPU processes)"
                         % (args.ngrads, world))


def build(args, rank=0, world=1, device=None):
    """Model + optimizer + trainer + actor-learner loop (+ callbacks) for this rank."""
    from .checkpoint import ModelSaver, PeriodicPerStepCallback, SaverRestore
    from .model import Model
    from .optimizer import SyncReplicasOptimizer, make_optimizer
    from .trainer import Ba3cTrainer, TrainConfig

    mc = model_config(args)
    seed = rank if args.seed is None else args.seed
    model = Model(conv_init=args.conv_init, fc_init=args.fc_init, seed=seed,
                  max_batch=max(args.batch_size, args.simulator_procs), **mc)
    oc = optimizer_config(args)
    opt = make_optimizer(oc["name"], oc["lr"], beta1=oc["beta1"], beta2=oc["beta2"],
                         epsilon=oc["epsilon"])
    if args.use_sync:
        opt = SyncReplicasOptimizer(opt, replicas_to_aggregate=args.ngrads, total_num_replicas=world)
    trainer = Ba3cTrainer(TrainConfig(model=model, optimizer=opt, step_per_epoch=args.steps_per_epoch,
                                      max_epoch=args.max_epoch))
    if args.load:
        SaverRestore(args.load).init(trainer)
        if isinstance(opt, SyncReplicasOptimizer):
            opt.broadcast_variables(trainer.engine)
    savers = []
    if args.save_every and rank == 0:
        savers.append(PeriodicPerStepCallback(ModelSaver(args.models_dir), args.save_every))
    return model, trainer, savers


class _Metrics(object):
    """DebugLogCallback over device-resident step scalars: each learner step's 8 scalars are
    kept on the GPU and fetched once per --send_debug_every steps (no per-step host sync)."""

    def __init__(self, trainer, batch_size, every, client):
        from .metrics import DebugLogCallback
        self.trainer, self.B = trainer, batch_size
        self.every = max(1, int(every))
        self.cb = DebugLogCallback(client, worker_id=0, nr_send=self.every) if client else None
        self.pending = []
        self.t0 = time.time()
        self.last = None

    def __call__(self, trainer):
        self.pending.append(trainer.model.scalars.clone())
        if len(self.pending) >= self.every:
            self.flush()

    def flush(self):
        if not self.pending:
            return
        from ._lib import SCALAR_NAMES
        vals = torch.stack(self.pending).cpu().numpy()
        self.trainer.check_device_errors()           # the host has synchronised anyway
        dt = time.time() - self.t0
        dp_per_s = len(self.pending) * self.B / max(dt, 1e-9)      # multigpu.py:307-313
        for row in vals:
            d = dict(zip(SCALAR_NAMES, row.tolist()))
            self.last = d
            if self.cb is not None:
                self.cb.trigger_step(d, dp_per_s)
        self.pending = []
        self.t0 = time.time()


def main(argv=None):
    args = resolve(build_parser().parse_args(argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    check_distributed(args, world)
    torch.cuda.set_device(local)
    own_group = False
    if args.use_sync and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
        own_group = True
    try:
        return _run(args, rank, world)
    finally:
        if own_group:
            dist.destroy_process_group()


def _run(args, rank, world):
    from .actor_learner import ActorLearner
    from .metrics import CsvChannels
    np.random.seed(rank)                                      # train.py:679
    model, trainer, savers = build(args, rank, world)
    client = CsvChannels(args.experiment_dir) if rank == 0 else None
    metrics = _Metrics(trainer, args.batch_size, args.send_debug_every, client)

    def on_step(tr):
        metrics(tr)
        for cb in savers:
            cb.trigger_step(tr)

    max_steps = args.max_steps or args.steps_per_epoch * args.max_epoch
    t0 = time.time()
    if args.dummy:
        # --dummy 1: a constant synthetic batch, no simulators (train/multigpu.py:70-75)
        dev = trainer.engine.device
        B = args.batch_size
        state = torch.ones(B, 84, 84, trainer.engine.channels, dtype=torch.uint8, device=dev)
        action = torch.zeros(B, dtype=torch.int64, device=dev)
        R = torch.zeros(B, dtype=torch.float32, device=dev)
        while trainer.global_step < max_steps:
            trainer.train_step(state, action, R)
            on_step(trainer)
        sim_steps = 0
    else:
        al = ActorLearner(trainer, n_envs=args.simulator_procs, batch_size=args.batch_size,
                          seed=rank, rs=np.random.RandomState(rank), on_train_step=on_step,
                          dummy_predictor=bool(args.dummy_predictor))
        while trainer.global_step < max_steps:
            al.iterate()
        sim_steps = al.steps
    metrics.flush()
    torch.cuda.synchronize()
    wall = time.time() - t0
    if client is not None:
        client.close()
    out = {"rank": rank, "world": world, "global_step": trainer.global_step,
           "simulator_steps": sim_steps, "samples_per_s": round(
               trainer.global_step * args.batch_size * world / max(wall, 1e-9), 1),
           "last": metrics.last}
    if rank == 0:
        print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
