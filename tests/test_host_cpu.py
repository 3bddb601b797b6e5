"""Host logic on CPU (no GPU): the trainer / SyncReplicasOptimizer aggregation over a
world-size-2 gloo group, the TF optimizer state bookkeeping and the flag surface.

The compute engine here is a test double backed by the oracle (test infrastructure); the
product path (Ba3cEngine) refuses to run without the HIP library and a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ba3c_oracle as O

CFG = {"fc_neurons": 16, "fc_splits": 2}


class OracleEngine(object):
    """Same surface as ba3c_amd.engine.Ba3cEngine, computing with the oracle on the CPU."""

    def __init__(self, params):
        self.names = list(params)
        self.shapes = {k: v.shape for k, v in params.items()}
        self.offs = {}
        off = 0
        for k in self.names:
            self.offs[k] = off
            off += params[k].size
        self.flat_size = off
        self.params = torch.from_numpy(np.concatenate([params[k].reshape(-1) for k in self.names]))
        self.grads = torch.zeros_like(self.params)
        self.scalars = torch.zeros(8, dtype=torch.float64)
        self.device = torch.device("cpu")
        self.num_actions = 4

    @property
    def tensor_names(self):
        return self.names

    @property
    def layout(self):
        return [(k, self.offs[k], int(np.prod(self.shapes[k])), self.shapes[k]) for k in self.names]

    def bucket_split(self):
        t = next(i for i, k in enumerate(self.names) if k.startswith("fc"))
        return t, self.offs[self.names[t]]

    def state_dict(self, flat=None):
        flat = (self.params if flat is None else flat).numpy()
        return {k: flat[self.offs[k]:self.offs[k] + int(np.prod(self.shapes[k]))].reshape(self.shapes[k]).copy()
                for k in self.names}

    def zeros_like_flat(self, fill=0.0):
        return torch.full((self.flat_size,), fill, dtype=torch.float32)

    def train_grads(self, state, action, R, entropy_beta=0.01, grads=None, phase=0):
        # phase 1 leaves the fc1 + heads bucket final, phase 2 the conv part (the HIP engine's
        # contract: each phase writes only its own bucket)
        _, off = self.bucket_split()
        if phase != 2:
            _, sc, g = O.loss_and_grads(self.state_dict(), state.numpy(), action.numpy(), R.numpy(), CFG)
            self._full = torch.from_numpy(np.concatenate([g[k].reshape(-1) for k in self.names]))
            self.scalars[0] = float(sc["cost"])
        if phase == 0:
            self.grads.copy_(self._full)
        elif phase in (1, 4):               # 4: phase 1 whose reduction the HIP engine holds
            self.grads[off:].copy_(self._full[off:])
        else:
            self.grads[:off].copy_(self._full[:off])
        return self.scalars

    def launch_held(self, stream=None):
        pass                                 # the held reduction: nothing to launch on the CPU

    def set_phase2_event(self, event):
        pass

    def clip_grads(self, grads=None):
        self.clip_grads_range(0, len(self.names))

    def clip_grads_range(self, t0, t1, grads=None, no_residency=False):
        g = self.state_dict(self.grads)
        for k in self.names[t0:t1]:
            n = int(np.prod(self.shapes[k]))
            self.grads[self.offs[k]:self.offs[k] + n].copy_(
                torch.from_numpy(O.clip_by_average_norm(g[k]).reshape(-1)))

    def apply_update(self, opt, slot0, slot1, hp, grad_scale=1.0, fuse_clip=False, grads=None,
                     dev_powers=None):
        assert opt == "adam"
        if fuse_clip:
            self.clip_grads()
            grad_scale = 1.0
        g = self.state_dict(self.grads)
        p, m, v = self.state_dict(), self.state_dict(slot0), self.state_dict(slot1)
        for k in self.names:
            gk = (g[k] * np.float32(grad_scale)).astype(np.float32)
            p[k], m[k], v[k] = O.apply_adam(p[k], gk, m[k], v[k], hp["lr"], hp["beta1"], hp["beta2"],
                                            hp["epsilon"], hp["beta1_power"], hp["beta2_power"])
        for buf, d in ((self.params, p), (slot0, m), (slot1, v)):
            buf.copy_(torch.from_numpy(np.concatenate([d[k].reshape(-1) for k in self.names])))


def _batch(seed, B=2):
    rs = np.random.RandomState(seed)
    return (rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8),
            rs.randint(0, 4, size=B).astype(np.int64), rs.normal(size=B).astype(np.float32))


# fixed arrival order per step for the backup-worker tests: ORDERS[step] lists ranks, first first
ORDERS = [[2, 0, 1], [1, 2, 0]]


def _fixed_arrival(rank, step):
    return float(ORDERS[step].index(rank))


def _worker(rank, world, port, out, bucketed=True, k=None, fixed=False, straggler=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time
    from ba3c_amd.model import Model
    from ba3c_amd.optimizer import AdamOptimizer, SyncReplicasOptimizer
    from ba3c_amd.trainer import Ba3cTrainer, TrainConfig
    params = O.init_params(16, 2, 4, seed=0, dtype=np.float32)
    eng = OracleEngine(params)
    model = Model(num_actions=4, fc_neurons=16, fc_splits=2, batch_size=2, engine=eng)
    opt = SyncReplicasOptimizer(AdamOptimizer(1e-3, 0.8, 0.75, 1e-8), k or world, world,
                                arrival_fn=_fixed_arrival if fixed else None)
    opt.bucketed = bucketed
    tr = Ba3cTrainer(TrainConfig(model=model, optimizer=opt))
    chosen = []
    for step in range(2):
        s, a, r = _batch(10 * step + rank)
        if straggler is not None and rank == straggler:
            time.sleep(1.5)                   # this replica's gradients arrive last
        tr.train_step(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(r))
        chosen.append(list(opt.last_aggregated))
    out[rank] = (eng.params.numpy().copy(), chosen, opt.dropped)
    dist.destroy_process_group()


def _oracle_sync(world, aggregate=None):
    params = O.init_params(16, 2, 4, seed=0, dtype=np.float32)
    slots = O.init_slots(params, "adam", 0.8, 0.75)
    for step in range(2):
        batches = [_batch(10 * step + r) for r in range(world)]
        params, slots, _, _ = O.train_step(params, slots, step + 1, batches, CFG, lr=1e-3,
                                           beta1=0.8, beta2=0.75, eps=1e-8,
                                           aggregate=None if aggregate is None else aggregate[step])
    return np.concatenate([params[k].reshape(-1) for k in params])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("bucketed", [True, False])
def test_sync_replicas_world2_gloo_matches_oracle_sync_step(bucketed):
    """Both exchanges — two buckets (fc1 + heads all-reduced beside the conv backward) and one
    flat all-reduce — equal the oracle's SyncReplicas step."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, bucketed), nprocs=world, join=True)
    # replicas stay bit-identical
    np.testing.assert_array_equal(out[0][0], out[1][0])
    # and equal the oracle's SyncReplicas step: mean of per-replica clipped grads, one Adam
    np.testing.assert_allclose(out[0][0], _oracle_sync(world), rtol=2e-6, atol=1e-9)


def test_backup_workers_aggregate_first_k_in_fixed_arrival_order():
    """num_grad=2 of 3 workers (train.py:601-602): each step the two first-arriving replicas'
    clipped grads are averaged, the third is dropped as stale; all replicas apply the same
    update and equal the oracle's mean over that subset."""
    world, k = 3, 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, True, k, True), nprocs=world, join=True)
    want = [sorted(o[:k]) for o in ORDERS]
    for r in range(world):
        np.testing.assert_array_equal(out[r][0], out[0][0])
        assert out[r][1] == want
        assert out[r][2] == sum(r not in w for w in want)
    np.testing.assert_allclose(out[0][0], _oracle_sync(world, want), rtol=2e-6, atol=1e-9)
    # dropping changes the update: the all-replica mean is a different point
    assert np.abs(out[0][0] - _oracle_sync(world)).max() > 1e-7


def test_backup_workers_drop_a_measured_straggler():
    """Measured arrival (host monotonic clock after the gradients are ready): a replica that
    sleeps 1.5 s before each step is the backup worker every step and its gradients never
    enter the mean."""
    world, k = 3, 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, True, k, False, 1), nprocs=world, join=True)
    for r in range(world):
        assert out[r][1] == [[0, 2], [0, 2]]
        np.testing.assert_array_equal(out[r][0], out[0][0])
    assert out[1][2] == 2
    np.testing.assert_allclose(out[0][0], _oracle_sync(world, [[0, 2], [0, 2]]),
                               rtol=2e-6, atol=1e-9)


def test_sync_replicas_validates_replica_counts():
    from ba3c_amd.optimizer import AdamOptimizer, SyncReplicasOptimizer
    with pytest.raises(ValueError):      # every rank is one replica: N must be the world size
        SyncReplicasOptimizer(AdamOptimizer(), replicas_to_aggregate=1, total_num_replicas=4)
    with pytest.raises(ValueError):      # cannot aggregate more replicas than exist
        SyncReplicasOptimizer(AdamOptimizer(), replicas_to_aggregate=2, total_num_replicas=1)
    assert SyncReplicasOptimizer(AdamOptimizer(), 1, 1).backup_workers == 0


def test_adam_beta_powers_follow_tf_float32_variables():
    from ba3c_amd.optimizer import AdamOptimizer
    o = AdamOptimizer(1e-3, beta1=0.8, beta2=0.75)
    hp0 = o._hparams()
    o._after_apply()
    o._after_apply()
    assert hp0["beta1_power"] == float(np.float32(0.8))
    assert o.beta1_power == np.float32(np.float32(np.float32(0.8) * np.float32(0.8)) * np.float32(0.8))
    assert o.beta2_power.dtype == np.float32


def test_flags_mirror_run_job():
    from ba3c_amd.flags import build_parser, resolve
    a = resolve(build_parser().parse_args(
        "-b 32 --fc_neurons 128 --fc_splits 4 -o adam --beta1 0.8 --beta2 0.75 --epsilon 1e-8 "
        "--use_sync -g 60 -l 0.001".split()))
    assert (a.batch_size, a.fc_neurons, a.fc_splits, a.optimizer, a.ngrads) == (32, 128, 4, "adam", 60)
    assert a.replace_with_conv is True
    a = resolve(build_parser().parse_args("--use_normal_fc --adam_debug --beta1 0.7".split()))
    assert a.replace_with_conv is False and a.beta2 == 0.7
    with pytest.raises(SystemExit):
        resolve(build_parser().parse_args(["--use_sync"]))


def test_product_engine_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ba3c_amd import Ba3cLibraryError
    from ba3c_amd.engine import Ba3cEngine
    with pytest.raises(Ba3cLibraryError):
        Ba3cEngine(num_actions=4, fc_neurons=128, fc_splits=4, max_batch=4)


def test_launcher_flags_build_the_reference_configuration():
    """`python -m ba3c_amd.train` reads run_job.py's flags into the model geometry, the
    optimizer and the sync-replica rule (train.py:582-606, run_job.py:13-57)."""
    from ba3c_amd.flags import build_parser, resolve
    from ba3c_amd.train import check_distributed, model_config, optimizer_config
    a = resolve(build_parser().parse_args(
        "-n 71 -g 2 -c 12 -o adam --use_sync -l 0.001 -b 32 --fc_neurons 128 --simulator_procs 10 "
        "--ps 4 --fc_splits 4 --epsilon 1e-8 --beta1 0.8 --beta2 0.75 -e Breakout-v0".split()))
    assert model_config(a) == dict(num_actions=4, channels=1, fc_neurons=128, fc_splits=4,
                                   replace_with_conv=True, ps=4, batch_size=32)
    assert optimizer_config(a) == dict(name="adam", lr=0.001, beta1=0.8, beta2=0.75, epsilon=1e-8)
    check_distributed(a, 2)
    check_distributed(a, 4)                  # -g 2 of 4: two backup workers (train.py:601-602)
    with pytest.raises(SystemExit):
        check_distributed(a, 1)              # cannot aggregate more gradients than processes
    a.ngrads = 0
    with pytest.raises(SystemExit):
        check_distributed(a, 4)
    b = resolve(build_parser().parse_args("-b 32 -o rms".split()))
    check_distributed(b, 1)
    with pytest.raises(SystemExit):
        check_distributed(b, 2)              # no asynchronous multi-GPU mode


def test_bench_prices_multi_job_launches_with_all_their_jobs():
    """bench.py roofline accounting: a multi-job launch (ba3c_kernel_merged) counts every job's
    algorithmic FLOPs, and its peak is the total over the time each job would take at its own
    path's peak (conv0's u8 x fp16 hi/lo at 2 products, conv1's fp16x3 at 3)."""
    import bench
    B = 2048
    macs = bench.layer_macs(4, 512)
    f, jobs = bench.probe_flops("conv0_wgrad", ["conv1_wgrad", "wgrad_reduce"], macs, B)
    assert jobs == ["conv0_wgrad", "conv1_wgrad"]
    assert f == 2.0 * (macs["conv0"] + macs["conv1"]) * B
    f1, j1 = bench.probe_flops("conv1_dgrad", [], macs, B)
    assert j1 == ["conv1_dgrad"] and f1 == 2.0 * macs["conv1"] * B
    assert bench.probe_flops("heads", [], macs, B)[0] is None
    t = 2.0 * macs["conv0"] * B / (bench.kernel_peak(2) * 1e12) + \
        2.0 * macs["conv1"] * B / (bench.kernel_peak(3) * 1e12)
    assert abs(f / t / 1e12 - 961.2) < 0.5          # the r03b line's combined peak


def _last_json(out):
    import json
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_spawns_its_own_ranks_without_torchrun():
    """`python bench.py --gpus 2` with no WORLD_SIZE (the driver's invocation) starts two rank
    processes itself — RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, a gloo group formed, the
    gradient-sized all-reduce summed — and rank 0 prints the one JSON line."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--exchange-selftest"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["sum_ok"] is True


def test_bench_spawner_returns_the_failing_rank_status(tmp_path):
    """A rank that dies makes the launcher stop the others after the grace period (a dead peer
    must not leave rank 0 waiting in a collective) and exit with the failing status."""
    import bench
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "assert os.environ['WORLD_SIZE'] == '3' and os.environ['LOCAL_RANK'] == str(r)\n"
                      "assert os.environ['MASTER_ADDR'] == '127.0.0.1'\n"
                      "if r == 1: sys.exit(3)\n"
                      "time.sleep(0 if r == 2 else 600)\n")
    import time
    t0 = time.time()
    rc = bench.spawn_ranks(3, [], script=str(script), grace=1.0)
    assert rc == 3, rc          # rank 1's own status, not rank 0's SIGKILL from the launcher
    assert time.time() - t0 < 60
    ok = tmp_path / "ok.py"
    ok.write_text("import os; assert os.environ['WORLD_SIZE'] == '2'\n")
    assert bench.spawn_ranks(2, [], script=str(ok), grace=1.0) == 0


def test_bench_spawner_deadline_kills_a_hung_job(tmp_path):
    """Ranks that never exit (a rank stuck inside a collective) are all killed at the overall
    deadline (BA3C_SPAWN_DEADLINE) and the launcher exits non-zero (124, as timeout(1))."""
    import time
    import bench
    script = tmp_path / "hang.py"
    script.write_text("import time\ntime.sleep(600)\n")
    t0 = time.time()
    rc = bench.spawn_ranks(2, [], script=str(script), grace=60.0, deadline=2.0)
    assert rc == bench.SPAWN_TIMEOUT_RC, rc
    assert time.time() - t0 < 30


def _replica_worker(rank, world, port, out, perturb):
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = torch.arange(1000, dtype=torch.float32) * 0.37
        m = torch.ones(1000)
        if perturb and rank == world - 1:
            m[517] = torch.nextafter(m[517], torch.tensor(2.0))   # one ulp on one rank
        out[rank] = bench.replicas_identical([p, m])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("perturb", [False, True])
def test_bench_replica_identity_check_world2(perturb):
    """bench.py's N>1 replica check: every rank agrees, and one ulp of
    difference in one slot of one rank makes every rank report False."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_replica_worker, args=(world, _free_port(), out, perturb), nprocs=world, join=True)
    assert out[0] == out[1] == (not perturb)


def test_bench_health_flags_make_the_run_fail():
    """bench.py writes ba3c_device_errors' flags into the line and returns a non-zero status
    for a non-zero flag or diverged replicas."""
    import bench
    out = {}
    assert bench.health(out, 0, None) == 0 and out["device_errors"] == 0
    out = {}
    assert bench.health(out, 2, True) == 1
    assert out["device_errors"] == 2 and "bucket clip" in out["device_errors_what"]
    assert out["replicas_identical"] is True
    out = {}
    assert bench.health(out, 0, False) == 1 and out["replicas_identical"] is False
