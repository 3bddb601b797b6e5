"""The bench workload's own kernels against the oracle, and the multi-replica / two-stream
paths of BASELINE configs[3] and configs[4] on one GPU.

* B=160 (C=4, F=512, S=1, A=4 — the bench geometry): B > SMALL_B = 128 selects the whole-map
  conv2 input-gradient kernel (L6Conv2D) and the conv2 forward of full bands, and 10*B > 512
  persistent workgroups makes conv0's weight gradient accumulate several bands per workgroup.
  Checked against the fp64 oracle evaluated in chunks of 16 (train.py:164-327,
  train/multigpu.py:85-86).
* B=256 vs 128: both conv2 geometries (L6Conv2D / L6Conv2F vs their small-batch 3-/2-row-band
  variants) give bit-identical activations and input gradients for the same images.
* The synchronous replica path (train.py:598-606, multigpu.py:157,194): per-replica clip, a
  sum of the clipped buffers, one update with grad_scale = 1/N and no fused clip; and the
  SyncReplicasOptimizer's RCCL all-reduce executed in a world-size-1 'nccl' process group.
* configs[4]: an 8192-state predictor forward on a second HIP stream concurrently with a
  B=2048 learner step equals the serial forward on the same parameter snapshot bit for bit
  (predict/concurrency.py:172-219, train.py:355-392).
"""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import ba3c_oracle as O
from test_gpu_parity import GRAD_TOL, FWD_TOL, as64, case, dev, engine, gpu_decisions, rel

pytestmark = pytest.mark.gpu


def test_bench_geometry_b160_matches_chunked_oracle():
    B = 160
    cfgk = dict(A=4, C=4, F=512, S=1)
    params, state, action, R, cfg = case(1600, B, wscale=2.0, **cfgk)
    eng = engine(max_batch=B, **cfgk)
    eng.load_params(params)
    sc = eng.train_grads(dev(state), dev(action), dev(R), entropy_beta=0.01)
    got = eng.state_dict(eng.grads)
    forced, codes = gpu_decisions(eng, B)
    t, osc, g = O.loss_and_grads_chunked(as64(params), state, action, R.astype(np.float64), cfg,
                                         forced=forced, chunk=16)
    for layer in range(3):
        assert np.mean(t["own_c%d" % layer] != codes[layer]) < 1e-4, layer
    assert np.mean(t["a3_pos"] != forced["a3_mask"]) < 1e-4
    for k in g:
        e = rel(got[k], g[k])
        assert e < GRAD_TOL, (k, e)
    assert np.all(got["conv0/W"][:, :, 4:, :] == 0)
    s = sc.cpu().numpy()
    from ba3c_amd._lib import SCALAR_NAMES
    for i, name in enumerate(SCALAR_NAMES[:7]):
        ref = float(osc[name])
        assert abs(s[i] - ref) <= 1e-4 * max(1.0, abs(ref)), (name, s[i], ref)
    assert abs(int(s[7]) - osc["active_relus"]) <= max(2, 1e-5 * osc["active_relus"])
    # the predictor forward of the same states at this batch
    probs, _, value = eng.forward(dev(state))
    assert rel(probs.cpu().numpy(), t["logits"]) < FWD_TOL


def test_conv2_geometries_are_bit_identical_across_small_batch_switch():
    """The same 128 images run once as a B=128 batch (2-/3-row-band conv2 kernels) and twice
    over as a B=256 batch (whole-map / full-band kernels).  The loss is a batch mean, so every
    backward value of the B=256 run is exactly half the B=128 one (1/256 = 1/128 / 2: powers of
    two commute with every rounding); activations are identical."""
    cfgk = dict(A=4, C=4, F=512, S=1)
    params, state, action, R, _ = case(129, 128, wscale=2.0, **cfgk)
    eng = engine(max_batch=256, **cfgk)
    eng.load_params(params)
    fwd_names, bwd_names = ("p1", "p2", "c1", "c2"), ("dp2", "dp1", "dp0")
    d = lambda x: dev(np.concatenate([x, x]))
    eng.train_grads(d(state), d(action), d(R))
    big = {n: eng.workspace_tensor(n, 256).clone() for n in fwd_names + bwd_names}
    eng.train_grads(dev(state), dev(action), dev(R))
    small = {n: eng.workspace_tensor(n, 128).clone() for n in fwd_names + bwd_names}
    torch.cuda.synchronize()
    for n in fwd_names + bwd_names:
        half = small[n].numel()
        want = small[n] if n in fwd_names else small[n] * 0.5
        assert torch.equal(big[n][:half], want), n
        assert torch.equal(big[n][half:], want), n


def _replica_batches(n, B, seed):
    out = []
    for r in range(n):
        rs = np.random.RandomState(seed + r)
        out.append((rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8),
                    rs.randint(0, 4, size=B).astype(np.int64), rs.normal(size=B).astype(np.float32)))
    return out


def test_sync_replica_update_path_matches_oracle_sync_step():
    """Two replicas on one GPU: each runs train_grads + clip_grads, the two flat buffers are
    summed (the RCCL sum's stand-in), and one apply_update(grad_scale=1/2, fuse_clip=0) follows
    — against the oracle's SyncReplicas step (mean of the per-replica clipped gradients, one
    TF Adam apply) from the same parameters and slots, for 2 consecutive steps."""
    from ba3c_amd.optimizer import AdamOptimizer
    cfgk = dict(A=4, C=4, F=128, S=4)
    params, _, _, _, cfg = case(77, 8, wscale=2.0, **cfgk)
    eng = engine(max_batch=16, **cfgk)
    eng.load_params(params)
    opt = AdamOptimizer(1e-3, beta1=0.8, beta2=0.75, epsilon=1e-8)
    for step in range(2):
        p0 = eng.state_dict()
        slots = {"m": {}, "v": {}, "beta1_power": opt.beta1_power, "beta2_power": opt.beta2_power}
        if opt.slots is not None:
            slots["m"], slots["v"] = eng.state_dict(opt.slots[0]), eng.state_dict(opt.slots[1])
        else:
            slots["m"] = {k: np.zeros_like(v) for k, v in p0.items()}
            slots["v"] = {k: np.zeros_like(v) for k, v in p0.items()}
        batches = _replica_batches(2, 8, 500 + 10 * step)
        total = torch.zeros_like(eng.grads)
        for (s, a, r) in batches:
            eng.train_grads(dev(s), dev(a), dev(r))
            eng.clip_grads()
            total += eng.grads
        eng.grads.copy_(total)
        opt.apply_gradients(eng, grad_scale=0.5, fuse_clip=False)
        got = eng.state_dict()
        s64 = {"m": as64(slots["m"]), "v": as64(slots["v"]),
               "beta1_power": slots["beta1_power"], "beta2_power": slots["beta2_power"]}
        newp, _, _, g = O.train_step(as64(p0), s64, step + 1,
                                     [(s, a, r.astype(np.float64)) for s, a, r in batches], cfg,
                                     lr=1e-3, beta1=0.8, beta2=0.75, eps=1e-8)
        for k in g:
            d_got = got[k].astype(np.float64) - p0[k]
            d_ref = newp[k] - p0[k]
            mask = np.abs(g[k]) > 1e-4 * max(np.abs(g[k]).max(), 1e-30)
            if mask.any():
                assert rel(d_got[mask], d_ref[mask]) < GRAD_TOL, (step, k)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("direct", ["1", "0"])
def test_sync_replicas_rccl_allreduce_world1_equals_single_replica_step(monkeypatch, direct):
    """SyncReplicasOptimizer inside a world-size-1 'nccl' (RCCL) process group: the clip, the
    RCCL all-reduce on the HIP stream and the grad_scale update run for real, and the result
    equals the single-replica fused-clip step bit for bit — with the bucket sums driven
    through RCCL directly (rccl.py, the default) and through torch's collective."""
    import torch.distributed as dist
    from ba3c_amd.model import Model
    from ba3c_amd.optimizer import AdamOptimizer, SyncReplicasOptimizer
    from ba3c_amd.trainer import Ba3cTrainer, TrainConfig
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    monkeypatch.setenv("BA3C_DIRECT_RCCL", direct)
    batches = [tuple(dev(x) for x in b) for b in _replica_batches(3, 16, 900)]
    opts = []

    def run(sync):
        m = Model(num_actions=4, fc_neurons=128, fc_splits=4, batch_size=16, max_batch=16, seed=9)
        opt = AdamOptimizer(1e-3, 0.8, 0.75, 1e-8)
        if sync:
            opt = SyncReplicasOptimizer(opt, replicas_to_aggregate=1, total_num_replicas=1)
            assert opt.distributed
            opts.append(opt)
        tr = Ba3cTrainer(TrainConfig(model=m, optimizer=opt))
        for b in batches:
            tr.train_step(*b)
        torch.cuda.synchronize()
        return m.engine.params.cpu().numpy()

    ref = run(False)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0,
                            world_size=1, device_id=torch.device("cuda", torch.cuda.current_device()))
    try:
        got = run(True)
        assert bool(opts[0]._rccl) == (direct == "1")
        if opts[0]._rccl:
            # what the N>1 line's exchange object records from every rank
            info = opts[0].rccl_info()
            assert info["comm_count"] == 1 and info["comm_user_rank"] == 0
            assert info["comm_device"] == torch.cuda.current_device()
            assert info["rccl_version"] > 0 and ":" in info["pci_bus_id"]
            assert opts[0]._rccl.selftest()
            opts[0].close()
            assert opts[0]._rccl is None
    finally:
        dist.destroy_process_group()
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("cu_mask", [None, 64])
def test_configs4_predictor_stream_beside_train_step_equals_serial(cu_mask):
    """configs[4] on one GPU: the learner (B=2048, F=512) and an 8192-state predictor forward
    on a second HIP stream reading a parameter snapshot taken on the learner stream (cu_mask:
    that stream restricted to 64 CUs, hipevent.CuMaskedStream, bench.py's partition variant).
    The overlapped predictor outputs equal a serial forward on that snapshot bit for bit, the
    learner's parameters equal a serial learner step's, and a 16-state slice matches the
    oracle."""
    from ba3c_amd import hipevent
    from ba3c_amd.engine import Ba3cEngine
    from ba3c_amd.model import Model
    from ba3c_amd.optimizer import AdamOptimizer
    from ba3c_amd.trainer import Ba3cTrainer, TrainConfig
    B, NP = 2048, 8192
    g = torch.Generator(device="cuda").manual_seed(44)
    state = torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device="cuda", generator=g)
    action = torch.randint(0, 4, (B,), dtype=torch.int64, device="cuda", generator=g)
    R = torch.randn(B, dtype=torch.float32, device="cuda", generator=g)
    sims = torch.randint(0, 256, (NP, 84, 84, 4), dtype=torch.uint8, device="cuda", generator=g)

    def learner():
        m = Model(num_actions=4, fc_neurons=512, fc_splits=1, batch_size=B, max_batch=B, seed=2)
        return Ba3cTrainer(TrainConfig(model=m, optimizer=AdamOptimizer(1e-3, 0.8, 0.75, 1e-8)))

    pe = Ba3cEngine(num_actions=4, fc_neurons=512, fc_splits=1, max_batch=NP)
    # serial reference: step 1, snapshot, forward, step 2
    ref = learner()
    ref.train_step(state, action, R)
    pe.params.copy_(ref.engine.params)
    want = [x.clone() for x in pe.forward(sims)]
    ref.train_step(state, action, R)
    torch.cuda.synchronize()

    tr = learner()
    tr.train_step(state, action, R)
    masked = hipevent.CuMaskedStream(cu_mask) if cu_mask else None
    main, side = torch.cuda.current_stream(), (masked.stream if masked else torch.cuda.Stream())
    pe.params.copy_(tr.engine.params)            # snapshot on the learner stream
    ev = torch.cuda.Event()
    ev.record(main)
    side.wait_event(ev)
    with torch.cuda.stream(side):
        got = pe.forward(sims)
    tr.train_step(state, action, R)              # concurrently on the learner stream
    main.wait_stream(side)
    torch.cuda.synchronize()
    for a, b in zip(got, want):
        assert torch.equal(a, b)
    assert torch.equal(tr.engine.params, ref.engine.params)
    snap = {k: v.astype(np.float64) for k, v in pe.state_dict().items()}
    t = O.get_nn_prediction(snap, sims[4000:4016].cpu().numpy(), {"fc_neurons": 512, "fc_splits": 1})
    assert rel(got[0][4000:4016].cpu().numpy(), t["logits"]) < FWD_TOL


def test_cabi_rccl_exchange_world1():
    """The C-ABI exchange (ba3c_comm_unique_id / ba3c_comm_init / ba3c_allreduce_sum / _mean,
    SURVEY.md §8b) in a world-1 communicator owned by the handle: the sum of exact small
    integers is exact, the mean over one rank is the identity, a second init on the same
    handle is refused, and destroy (plain and abort) leaves the handle usable for a new one."""
    import ctypes
    from ba3c_amd import _lib
    from ba3c_amd.engine import Ba3cEngine
    eng = Ba3cEngine(num_actions=4, fc_neurons=128, fc_splits=4, max_batch=4)
    lib = eng.lib
    uid = ctypes.create_string_buffer(128)
    _lib.check(lib.ba3c_comm_unique_id(uid))
    _lib.check(lib.ba3c_comm_init(eng.h, uid, 1, 0))
    assert lib.ba3c_comm_init(eng.h, uid, 1, 0) != 0          # one communicator per handle
    n = 100003
    x = torch.arange(n, dtype=torch.float32, device="cuda")
    want = x.clone()
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.ba3c_allreduce_sum(eng.h, stream, ctypes.c_void_p(x.data_ptr()), n))
    _lib.check(lib.ba3c_allreduce_mean(eng.h, stream, ctypes.c_void_p(x.data_ptr()), n))
    torch.cuda.synchronize()
    assert torch.equal(x, want)
    _lib.check(lib.ba3c_comm_destroy(eng.h, 0))
    assert lib.ba3c_allreduce_sum(eng.h, stream, ctypes.c_void_p(x.data_ptr()), n) != 0
    _lib.check(lib.ba3c_comm_unique_id(uid))
    _lib.check(lib.ba3c_comm_init(eng.h, uid, 1, 0))
    _lib.check(lib.ba3c_comm_destroy(eng.h, 1))


def test_probe_every_brackets_one_launch_in_n():
    """ba3c_probe_every (bench.py --probe-every): the probe brackets the first of every n
    launches of its kernel from ba3c_probe_enable on; probe_enable(None) restores n = 1."""
    B = 32
    cfgk = dict(A=4, C=4, F=128, S=4)
    params, state, action, R, cfg = case(77, B, **cfgk)
    eng = engine(max_batch=B, **cfgk)
    eng.load_params(params)
    args = (dev(state), dev(action), dev(R))
    for every, steps, want in ((1, 4, 4), (3, 7, 3), (5, 5, 1)):
        eng.probe_enable("conv1_fwd", every)
        for _ in range(steps):
            eng.train_grads(*args)
        ms, n = eng.probe_read()
        assert n == want and ms > 0, (every, steps, n, ms)
    eng.probe_enable(None)
    with pytest.raises(RuntimeError):
        _lib_check_every(eng, 0)


def _lib_check_every(eng, n):
    from ba3c_amd import _lib
    _lib.check(eng.lib.ba3c_probe_every(eng.h, n))
