"""BA3C train-step throughput on MI355X (BASELINE.json metric).

One step = forward + A3C loss + backward + per-tensor clip + (RCCL gradient mean for N>1) +
Adam, on a synthetic 84x84x4 uint8 frame batch already resident in HBM.  Default workload:
configs[2]/[3] — B=2048 per GPU, fc_neurons=512, fc_splits=1, A=4 (Breakout), Adam with the
README's best hyper-parameters.  The B=32 / F=128 / S=4 parity configuration (configs[1]) is
timed beside it.  Rank 0 prints ONE JSON line.

    python bench.py --gpus N --steps K --warmup W     (N > 1: starts N rank processes itself)
    torchrun --nproc-per-node N ... bench.py --gpus N   (one process per GPU, RCCL)

Without WORLD_SIZE in the environment and --gpus N > 1, this process is only a launcher: it
makes no GPU call, starts N children (`python bench.py ...` with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, one per GPU), lets rank 0 print the
line and exits with the worst child's status.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-ba3c_amd"))
sys.path.insert(0, ROOT)

from ba3c_amd import hipevent  # noqa: E402  (HIP events without a system fence)

METRIC = "BA3C train-step samples/sec, 84x84x4 frames, batch 32 & 2048, at 1/2/4/8 GPUs"
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix peak (spec)
BF16_MFMA_PEAK_TFLOPS = 2516.6  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 (16 x the fp32 rate)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def kernel_peak(split):
    """Ceiling of a kernel in algorithmic fp32 TFLOP/s given its arithmetic path: fp32 MFMA,
    or a bf16 split issuing `split` bf16 products per fp32 product (ba3c_kernel_split)."""
    return FP32_MFMA_PEAK_TFLOPS if split <= 1 else BF16_MFMA_PEAK_TFLOPS / split


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary
    (scripts/pmc_summary.py: 2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of
    MI355X_MICROARCH.md §HBM), or None if it was not collected for this kernel."""
    try:
        d = json.load(open(PMC_TRAFFIC))
    except (OSError, ValueError):
        return None
    k = d.get("kernels", {}).get(kernel)
    return None if k is None or "hbm_bytes" not in k else int(k["hbm_bytes"])

# algorithmic MAC per sample of each layer's forward product (real C input channels;
# SURVEY.md §8d), backward kernels of a layer do the same algorithmic work
def layer_macs(C, F):
    return {"conv0": 6400 * 32 * 25 * C, "conv1": 1296 * 32 * 800, "conv2": 196 * 64 * 800,
            "conv3": 25 * 64 * 576, "fc1": 1600 * F}


KERNEL_LAYER = {"conv0_fwd": "conv0", "conv1_fwd": "conv1", "conv2_fwd": "conv2",
                "conv3_fwd": "conv3", "fc1_fwd": "fc1", "conv1_dgrad": "conv1",
                "conv2_dgrad": "conv2", "conv3_dgrad": "conv3", "fc1_dgrad": "fc1",
                "conv0_wgrad": "conv0", "conv1_wgrad": "conv1", "conv2_wgrad": "conv2",
                "conv3_wgrad": "conv3", "fc1_wgrad": "fc1"}


def probe_flops(dom, merged, macs, B):
    """Algorithmic FLOPs of one launch of the probed kernel id, including the kernels that ran
    inside the same multi-job launch (`merged`, from ba3c_kernel_merged: they record no launch
    of their own)."""
    jobs = [dom] + [k for k in merged if k in KERNEL_LAYER]
    if any(k not in KERNEL_LAYER for k in jobs):
        return None, jobs
    return sum(2.0 * macs[KERNEL_LAYER[k]] * B for k in jobs), jobs


def train_step_flops(B, C, F, A=4):
    """fwd + wgrad(all) + dgrad(all but conv0), real input channels."""
    m = layer_macs(C, F)
    fwd = sum(m.values())
    return 2.0 * (fwd + fwd + (fwd - m["conv0"])) * B


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SPAWN_TIMEOUT_RC = 124          # every rank killed at the overall deadline (as timeout(1))


def spawn_ranks(n, argv, script=None, grace=None, deadline=None):
    """`python bench.py --gpus N` without torchrun: start N rank processes of `script` (this
    file) with the environment torchrun would give them (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT), one per local GPU.  This
    process makes no GPU call; the children inherit stdout (rank 0 prints the JSON line).

    Two guards, so a hung job ends before the driver's limit: if a rank fails, the others get
    `grace` seconds (BA3C_SPAWN_GRACE, default 60) to end before they are killed (a dead peer
    cannot leave rank 0 waiting in a collective); and if the job is still running `deadline`
    seconds after the start (BA3C_SPAWN_DEADLINE, default 900) every rank is killed — a rank
    stuck inside a collective never exits, so the grace timer alone would never start.
    Returns the status of the FIRST rank seen to fail (a signal s counts as 128 + s), not the
    status of the peers this launcher killed afterwards; SPAWN_TIMEOUT_RC (124) at the
    deadline; 0 when every rank succeeded."""
    import signal
    import subprocess
    if grace is None:
        grace = float(os.environ.get("BA3C_SPAWN_GRACE", "60"))
    if deadline is None:
        deadline = float(os.environ.get("BA3C_SPAWN_DEADLINE", "900"))
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)]
                                      + list(argv), env=env))

    def stop(signum, frame):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        raise SystemExit(128 + signum)

    def status(rc):
        return 128 - rc if rc < 0 else rc

    old = {s: signal.signal(s, stop) for s in (signal.SIGTERM, signal.SIGINT)}
    t_start = time.time()
    first_rc, timed_out = None, False
    try:
        failed_at = None
        while True:
            rcs = [p.poll() for p in procs]
            if all(rc is not None for rc in rcs):
                break
            if first_rc is None:
                bad = [rc for rc in rcs if rc not in (None, 0)]
                if bad:
                    first_rc, failed_at = status(bad[0]), time.time()
            now = time.time()
            if (failed_at is not None and now - failed_at > grace) or now - t_start > deadline:
                if failed_at is None:
                    timed_out = True
                    print("bench: ranks still running %.0f s after the start "
                          "(BA3C_SPAWN_DEADLINE); killing all" % deadline, file=sys.stderr,
                          flush=True)
                for p in procs:
                    if p.poll() is None:
                        p.kill()
                for p in procs:
                    p.wait()
                continue
            time.sleep(0.1)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    if first_rc is not None:
        return first_rc
    if timed_out:
        return SPAWN_TIMEOUT_RC
    bad = [status(rc) for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def exchange_selftest(world, rank, iters=5):
    """--exchange-selftest: the launcher and process group without a GPU — each rank sums a
    gradient-sized fp32 buffer (0.95 M floats, F=512) over gloo on the CPU; rank 0 prints one
    JSON line (CPU test of the spawner, tests/test_host_cpu.py)."""
    dist.init_process_group("gloo")
    n = 948229
    x = torch.full((n,), float(rank + 1))
    ts = []
    for _ in range(iters):
        x.fill_(float(rank + 1))
        t0 = time.perf_counter()
        dist.all_reduce(x)
        ts.append(time.perf_counter() - t0)
    ok = bool(torch.all(x == world * (world + 1) / 2.0))
    el = torch.tensor([float(np.median(ts))], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "selftest": "gloo all-reduce of %d fp32 on the CPU"
                          % n, "n_gpus": world, "sum_ok": ok,
                          "allreduce_ms": round(float(el[0]) * 1000.0, 3)}), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


def build_trainer(B, F, S, A, world, seed, sync=False):
    from ba3c_amd.model import Model
    from ba3c_amd.optimizer import AdamOptimizer, SyncReplicasOptimizer
    from ba3c_amd.trainer import Ba3cTrainer, TrainConfig

    # reference initialisers (conv2d.py:48-55, fc.py:35-38) from the product package, seed 0
    model = Model(num_actions=A, channels=1, fc_neurons=F, fc_splits=S, batch_size=B, max_batch=B,
                  seed=0)
    opt = AdamOptimizer(1e-3, beta1=0.8, beta2=0.75, epsilon=1e-8)   # README.md:35
    if world > 1 or sync:
        # every rank's gradients enter every step's mean (no backup workers in the bench)
        opt = SyncReplicasOptimizer(opt, replicas_to_aggregate=world, total_num_replicas=world)
    tr = Ba3cTrainer(TrainConfig(model=model, optimizer=opt))
    g = torch.Generator(device="cuda").manual_seed(1000 + seed)
    state = torch.randint(0, 256, (B, 84, 84, 4), dtype=torch.uint8, device="cuda", generator=g)
    action = torch.randint(0, A, (B,), dtype=torch.int64, device="cuda", generator=g)
    R = torch.randn(B, dtype=torch.float32, device="cuda", generator=g)
    return tr, (state, action, R)


def sync_all(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()


def time_steps(tr, batch, steps, warmup, world, probe=None, probe_every=1):
    """Time exactly `steps` steps bracketed by barrier + synchronize (max over ranks): the
    wall clock, and HIP events around the whole run on the learner stream.  Then, outside the
    timed region, `steps` more steps with an event after each (every event recorded on the
    learner stream leaves a 5-6 us gap between its kernels, r06c trace) for the per-step
    median.  `probe`: the kernel whose launches the HIP-event probe brackets inside the timed
    steps, the first of every `probe_every` (each bracket's two events leave ~10 us of gaps in
    the stream, so a throughput run samples them; ba3c_probe_every)."""
    for _ in range(warmup):
        tr.train_step(*batch)
    sync_all(world)
    if probe is not None:
        tr.engine.probe_enable(probe, probe_every)   # the dominant kernel, timed steps only
    e0, e1 = hipevent.timing_event(), hipevent.timing_event()   # no system fence (hipevent.py)
    t0 = time.perf_counter()
    e0.record()
    for i in range(steps):
        tr.train_step(*batch)
    e1.record()
    sync_all(world)
    wall = time.perf_counter() - t0
    gpu_s = e0.elapsed_time(e1) / 1000.0
    probe_ms, launches = 0.0, 0
    if probe is not None:
        probe_ms, launches = tr.engine.probe_read()   # the probe covers the timed steps only
        tr.engine.probe_enable(None)
    evs = [hipevent.timing_event() for _ in range(steps + 1)]
    evs[0].record()
    for i in range(steps):
        tr.train_step(*batch)
        evs[i + 1].record()
    sync_all(world)
    per_step = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
    el = torch.tensor([max(wall, gpu_s), float(np.median(per_step))], dtype=torch.float64,
                      device="cuda")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    return float(el[0].item()), float(el[1].item()), probe_ms, launches


def time_graph_steps(tr, batch, steps, warmup):
    """Single-GPU small-batch step replayed as one captured hipGraph per step."""
    replay = tr.capture_step(*batch)
    for _ in range(warmup):
        replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        replay()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def overlap_bench(tr, batch, pred_batch, iters, world, masks=(64, 128)):
    """configs[4]: predictor forward of `pred_batch` simulator states on a second HIP stream
    beside the train step.  The predictor engine reads a parameter snapshot taken at the start
    of each iteration (stricter than the reference's Hogwild reads).  Both sides
    fill every CU, so the predictor can only gain where the learner leaves CUs idle; `masks`:
    the same with the predictor's stream restricted to that many CUs (CuMaskedStream), so its
    workgroups cannot displace the learner's on the other CUs."""
    from ba3c_amd.engine import Ba3cEngine
    eng = tr.engine
    pe = Ba3cEngine(num_actions=eng.num_actions, channels=eng.channels,
                    fc_neurons=eng.cfg["fc_neurons"], fc_splits=eng.cfg["fc_splits"],
                    max_batch=pred_batch)
    g = torch.Generator(device="cuda").manual_seed(4242)
    states = torch.randint(0, 256, (pred_batch, 84, 84, eng.channels), dtype=torch.uint8,
                           device="cuda", generator=g)
    ps = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    masked = {k: hipevent.CuMaskedStream(k) for k in masks}

    def pred_only():
        pe.params.copy_(eng.params)
        pe.forward(states)

    def run(mode, n, ps=ps):
        sync_all(world)
        t0 = time.perf_counter()
        for _ in range(n):
            if mode in ("train", "both"):
                if mode == "both":
                    pe.params.copy_(eng.params)          # snapshot on the learner stream
                    ev = hipevent.join_event()
                    ev.record(main)
                tr.train_step(*batch)
            if mode == "pred":
                pred_only()
            if mode == "both":
                if isinstance(ev, hipevent.HipEvent):
                    ev.wait(ps)
                else:
                    ps.wait_event(ev)
                with torch.cuda.stream(ps):
                    pe.forward(states)
                hipevent.wait_stream(main, ps)
        sync_all(world)
        return (time.perf_counter() - t0) / n * 1000.0

    run("both", 2)
    t_train = run("train", iters)
    t_pred = run("pred", iters)
    t_both = run("both", iters)
    part = {}
    for k, ms in masked.items():
        run("both", 2, ms.stream)
        part["predictor_on_%d_cus" % k] = round(run("both", iters, ms.stream), 4)
    B = batch[0].shape[0]
    return {"config": "configs[4]: predictor forward of %d states/GPU + train step (B=%d) on "
                      "separate HIP streams" % (pred_batch, B),
            "train_ms": round(t_train, 4), "predict_ms": round(t_pred, 4),
            "overlapped_ms": round(t_both, 4),
            "overlap_speedup": round((t_train + t_pred) / t_both, 3),
            "cu_masked_overlapped_ms": part,
            "cu_masked_speedup": {k: round((t_train + t_pred) / v, 3) for k, v in part.items()},
            "predict_states_per_s": round(world * pred_batch / (t_pred / 1000.0), 1)}


# launches of the second backward phase, which run beside the fc1 + heads bucket's all-reduce
PHASE2_KERNELS = ("conv3_dgrad", "conv3_wgrad", "conv2_dgrad", "conv1_dgrad", "conv0_wgrad",
                  "wgrad_reduce")


def occupy_table(tr, batch, ks, window_us, phase2_us, iters, world, probe, base):
    """--occupy: for each K, a launch on the exchange stream holds K CUs (ba3c_occupy_cus)
    right after the fc1 + heads bucket's sum, first for `window_us` (about the bucket's sum on
    an 8-GPU node) then for the whole of phase 2 (`phase2_us`, the worst case: CUs missing
    during every phase-2 launch).  Each row: the step time over `iters` steps and every
    phase-2 launch's time, against `base` (the same launches with the exchange running and no
    occupier) — `ideal` is what a perfectly balanced launch would take with K of the CUs gone
    for its whole length (base x CUs / (CUs - K)); a static per-CU partition of work instead
    waits for the occupier before its displaced workgroups start."""
    opt = tr.optimizer
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    rows = []
    try:
        for k in ks:
            for mode, us in (("window", window_us), ("phase2", phase2_us)):
                opt.occupy = (k, us)
                sync_all(world)
                ev = [hipevent.timing_event() for _ in range(2)]
                ev[0].record()
                for _ in range(iters):
                    tr.train_step(*batch)
                ev[1].record()
                sync_all(world)
                step = ev[0].elapsed_time(ev[1]) / iters
                launches = {kk: probe(kk) for kk in PHASE2_KERNELS}
                rows.append({"cus_held": k, "mode": mode, "hold_us": round(us, 1),
                             "step_ms": round(step, 4),
                             "launch_ms": {kk: round(v, 4) for kk, v in launches.items()},
                             "slowdown": {kk: round(v / base[kk], 3) if base.get(kk) else None
                                          for kk, v in launches.items()},
                             "ideal_slowdown_full_overlap": round(cus / (cus - k), 3)})
    finally:
        opt.occupy = None
    return rows


def exchange_report(tr, batch, iters, world, occupy=(), occupy_us=50.0):
    """N > 1 (or --sync-path): where the data-parallel exchange's time goes.  After the timed
    region, `iters` real bucketed steps record HIP events inside the step (ExchangeTimeline:
    phase 1, phase 2, the exchange stream's start after the phase-2 event, each bucket's
    all-reduce, the exposed wait, the update); every field is the max over ranks.  The marks
    are kept out of the timed steps: each event recorded on the learner stream costs a
    5-6 us gap between its kernels (r06c trace), so `timeline.step_ms` includes about seven of
    them.  Then each phase-2 launch is probed over `iters` steps with the exchange running
    and with it left out (each rank applies its own gradients; replicas diverge from here),
    so the cost of RCCL sharing CUs with the persistent conv kernels shows per launch."""
    from ba3c_amd.trainer import ExchangeTimeline
    opt, eng = tr.optimizer, tr.engine
    timeline = ExchangeTimeline()
    tr.timeline = timeline
    sync_all(world)
    for _ in range(iters):
        tr.train_step(*batch)
    sync_all(world)
    tr.timeline = None
    tb, off = eng.bucket_split()
    rccl_comms = None
    if dist.is_initialized():
        info = opt.rccl_info() if hasattr(opt, "rccl_info") else None
        if info is not None:
            info["torch_device"] = torch.cuda.current_device()
        rccl_comms = [None] * dist.get_world_size()
        dist.all_gather_object(rccl_comms, info)
    total = eng.grads.numel()
    tl = timeline.summary()
    names = sorted(k for k in tl if k.endswith("_ms"))

    def probe(k):
        eng.probe_enable(k)
        for _ in range(iters):
            tr.train_step(*batch)
        ms, n = eng.probe_read()
        eng.probe_enable(None)
        return ms / max(n, 1)

    tr.timeline = None
    sync_all(world)
    with_x = {k: probe(k) for k in PHASE2_KERNELS}
    was, opt.distributed = opt.distributed, False
    try:
        local = {k: probe(k) for k in PHASE2_KERNELS}
    finally:
        opt.distributed = was
    vals = [tl[k] for k in names] + [with_x[k] for k in PHASE2_KERNELS] + \
        [local[k] for k in PHASE2_KERNELS]
    el = torch.tensor(vals, dtype=torch.float64, device="cuda")
    if dist.is_initialized():
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = el.tolist()
    tl.update({k: round(v, 4) for k, v in zip(names, el[:len(names)])})
    n = len(PHASE2_KERNELS)
    occ = None
    if occupy:
        base = dict(zip(PHASE2_KERNELS, el[len(names):len(names) + n]))
        occ = occupy_table(tr, batch, occupy, occupy_us, tl["phase2_ms"] * 1000.0, iters, world,
                           probe, base)
    return {"buckets": {"fc1_heads": {"bytes": 4 * (total - off)}, "conv": {"bytes": 4 * off}},
            "backend": dist.get_backend() if dist.is_initialized() else None,
            # bucket sums through RCCL driven directly (rccl.py) or torch's collective
            "collective": "rccl-direct" if getattr(opt, "_rccl", None) else "torch",
            "timeline": tl,
            "phase2_launch_ms": {k: {"with_exchange": round(a, 4), "exchange_off": round(b, 4)}
                                 for k, a, b in zip(PHASE2_KERNELS, el[len(names):len(names) + n],
                                                    el[len(names) + n:])},
            "probe_iters": iters,
            "occupy": occ,
            # what RCCL itself reports on every rank (rank count, own rank, HIP device, PCI
            # bus id): world ranks on world distinct devices
            "rccl_comms": rccl_comms}


def find_dominant_kernel(tr, batch, steps=5, warm=20):
    """Probe every kernel id over `steps` steps: (the id with the longest launch time per
    step, {id: ms per step}).  A multi-job launch is timed under its job 0's id; the other
    jobs' ids read 0 (ba3c_kernel_merged lists them).  `warm` steps first: the clock is still
    ramping over the first steps after start (r06b: conv0 and conv1's forward, the first ids
    probed, read 46 and 58 us above their rocprofv3 medians after 2 warm steps)."""
    from ba3c_amd._lib import KERNEL_IDS
    eng = tr.engine
    for _ in range(warm):
        tr.train_step(*batch)
    best, best_ms, per = None, -1.0, {}
    for name in KERNEL_IDS:
        eng.probe_enable(name)
        for _ in range(steps):
            tr.train_step(*batch)
        ms, n = eng.probe_read()
        ms /= steps
        per[name] = ms
        if ms > best_ms:
            best, best_ms = name, ms
    eng.probe_enable(None)
    return best, per


def step_ceiling(eng, per_kernel, B, C, F):
    """The step against its real ceiling: every matrix launch's algorithmic FLOPs at the peak
    of the arithmetic path it runs on (ba3c_kernel_split: fp16x3 838.9, u8 x fp16x2 1258,
    bf16x6 419.4 TF/s), summed = the ideal step time of the mixed path; and the conv layers'
    time-weighted fraction (ideal / measured over the conv0..conv3 launches, a multi-job
    launch counted with all its jobs under job 0's time).  Elementwise / reduction launches
    (heads, reductions, clip, update) are not in the ideal."""
    macs = layer_macs(C, F)
    ideal = {}
    for k, layer in KERNEL_LAYER.items():
        ideal[k] = 2.0 * macs[layer] * B / (kernel_peak(eng.kernel_split(k)) * 1e12) * 1e3
    conv_ideal = conv_meas = 0.0
    for k, ms in per_kernel.items():
        if k not in KERNEL_LAYER or ms <= 0:
            continue
        jobs = [k] + [j for j in eng.kernel_merged(k) if j in KERNEL_LAYER]
        if KERNEL_LAYER[k].startswith("conv"):
            conv_ideal += sum(ideal[j] for j in jobs)
            conv_meas += ms
    return {"ideal_ms": round(sum(ideal.values()), 4),
            "conv_ideal_ms": round(conv_ideal, 4), "conv_measured_ms": round(conv_meas, 4),
            "conv_frac_time_weighted": round(conv_ideal / conv_meas, 4) if conv_meas else None}


def cpu_threads():
    """Threads the CPU baseline may use: the process's CPU share (OMP_NUM_THREADS on the GPU
    box, else the CPUs this process may run on)."""
    n = os.environ.get("OMP_NUM_THREADS")
    if n and n.isdigit() and int(n) > 0:
        return int(n)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def cpu_baseline(F, S, A, big_seconds=10.0, b32_steps=50):
    """SURVEY.md §8d / BASELINE.md §2: the PyTorch-CPU fp32 restatement of the reference TF
    graph (oracle/ba3c_torch_cpu.py: 16-channel padding, log-eps loss, autodiff, TF clip, TF
    Adam) timed on this host's cores beside the GPU: the bench workload (B=2048, F, S) for a
    bounded number of steps (>= 2, ~`big_seconds`) and configs[1] (B=32, F=128, S=4) for
    `b32_steps` steps; median step time of each."""
    from oracle import ba3c_oracle as O
    from oracle.ba3c_torch_cpu import TorchCpuBa3c
    threads = cpu_threads()
    torch.set_num_threads(threads)

    def run(B, F_, S_, min_steps, max_steps, seconds, warm):
        rs = np.random.RandomState(0)
        m = TorchCpuBa3c(O.init_params(F_, S_, A, seed=0, dtype=np.float32), F_, S_)
        st = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8))
        ac = torch.from_numpy(rs.randint(0, A, size=B).astype(np.int64))
        R = torch.from_numpy(rs.normal(size=B).astype(np.float32))
        for _ in range(warm):
            m.step(st, ac, R)
        ts = []
        t_all = time.perf_counter()
        while len(ts) < max_steps and (len(ts) < min_steps or time.perf_counter() - t_all < seconds):
            t0 = time.perf_counter()
            m.step(st, ac, R)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), len(ts)

    big_med, big_n = run(2048, F, S, 5, 20, big_seconds, 1)
    small_med, small_n = run(32, 128, 4, b32_steps, b32_steps, 0.0, 3)
    return {"value": round(2048 / big_med, 2), "unit": "samples/s", "cores": threads,
            "kind": "port",
            "sample": "PyTorch-CPU fp32 restatement of the reference TF graph (oracle/ba3c_torch_cpu.py),"
                      " %d threads on %s: B=2048 F=%d S=%d median of %d steps (%.2f s/step); "
                      "configs[1] B=32 F=128 S=4 median of %d steps" % (
                          threads, cpu_model(), F, S, big_n, big_med, small_n),
            "b32_value": round(32 / small_med, 2), "b32_ms_per_step": round(small_med * 1000, 2)}


def replicas_identical(tensors, group=None):
    """N > 1: every rank's tensors (parameters, optimizer slots) equal rank 0's bit for bit —
    the synchronous step's invariant (identical update on identical sums).  Rank 0's copies are
    broadcast and compared on every rank; the verdict is agreed with a MIN all-reduce, so all
    ranks return the same bool."""
    ok = True
    for t in tensors:
        ref = t.clone()
        dist.broadcast(ref, src=0, group=group)
        ok = ok and bool(torch.equal(ref, t))
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=tensors[0].device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item())


def health(out, flags, identical=None):
    """Write the run's health into the line: the engine's device error flags after the timed
    steps (ba3c_device_errors: an in-launch wait that gave up makes the parameters invalid)
    and, for N > 1, whether the replicas stayed bit-identical.  Returns the process status:
    non-zero when either check failed, so a wrong run cannot pass as a valid line."""
    from ba3c_amd.trainer import Ba3cTrainer
    out["device_errors"] = int(flags)
    if flags:
        out["device_errors_what"] = Ba3cTrainer.describe_device_errors(flags)
    if identical is not None:
        out["replicas_identical"] = bool(identical)
    return 1 if flags or identical is False else 0


ARITH = ("fp32-class products on 16-bit MFMA with fp32 accumulation: conv0 u8 x fp16 hi/lo "
         "(2 products), conv0..conv3 power-of-two-scaled fp16 hi/lo (3 products: hi*hi + hi*lo "
         "+ lo*hi), fc1 / heads weight gradient bf16 hi/mid/lo (6 products); per product ~2^-20 "
         "relative (fp32 rounding 2^-24), normwise per tensor; elements below ~2^-17 of their "
         "image's / tensor's max |x| lose fp16 bits (DESIGN.md §3.1)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    # the roofline probe brackets the dominant launch of one timed step in this many (1: every
    # step; one in 5 measured the same step time, r06s)
    ap.add_argument("--probe-every", type=int, default=1)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--fc_neurons", type=int, default=512)
    ap.add_argument("--fc_splits", type=int, default=1)
    ap.add_argument("--num_actions", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-b32", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--predict_batch", type=int, default=8192)
    ap.add_argument("--cpu-seconds", type=float, default=30.0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, one GPU per rank); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--sync-path", action="store_true",
                    help="N=1: run the N>1 step (SyncReplicasOptimizer: phase-split backward, "
                         "per-bucket clip, unfused update) in a world-1 RCCL group")
    ap.add_argument("--occupy", default="",
                    help="with --sync-path or N>1: comma-separated CU counts K; for each, a launch "
                         "on the exchange stream holds K CUs after the fc1 bucket's sum (for "
                         "--occupy-us, and for the whole of phase 2) and the line's "
                         "exchange.occupy table reports the step and every phase-2 launch")
    ap.add_argument("--occupy-us", type=float, default=50.0,
                    help="the short occupancy window (microseconds) of --occupy")
    ap.add_argument("--exchange-selftest", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launcher only: no GPU call in this process (the children set their devices)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    if args.exchange_selftest:
        sys.exit(exchange_selftest(world, rank))
    sys.exit(run_rank(args, world, rank, local))


def run_rank(args, world, rank, local):
    if args.dist_backend == "gloo":
        # rehearsal of N ranks on fewer GPUs: the exchange goes through a host copy
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    sync = world > 1 or args.sync_path
    if sync:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        if args.dist_backend == "gloo":
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))

    B, F, S, A = args.batch, args.fc_neurons, args.fc_splits, args.num_actions
    C = 4
    tr, batch = build_trainer(B, F, S, A, world, seed=rank, sync=sync)
    for _ in range(2):
        tr.train_step(*batch)
    sync_all(world)
    dom, per_kernel = find_dominant_kernel(tr, batch)
    ceiling = step_ceiling(tr.engine, per_kernel, B, C, F)
    # A/B runs: time a named kernel over the timed steps instead of the dominant one
    dom = os.environ.get("BA3C_BENCH_PROBE", dom)
    sync_all(world)

    elapsed, med_ms, probe_ms, launches = time_steps(tr, batch, args.steps, args.warmup, world,
                                                     probe=dom, probe_every=args.probe_every)
    flags = tr.engine.device_errors()     # synchronises; after the timed region
    identical = None
    if world > 1:
        inner = tr.optimizer._opt if hasattr(tr.optimizer, "_opt") else tr.optimizer
        identical = replicas_identical([tr.engine.params] + list(inner.slots or []))

    value = world * B * args.steps / elapsed
    ms_step = elapsed / args.steps * 1000.0
    macs = layer_macs(C, F)
    dom_flops, dom_jobs = probe_flops(dom, tr.engine.kernel_merged(dom), macs, B)
    # a multi-job launch's ceiling: its total FLOPs over the time every job would take at the
    # peak of its own arithmetic path
    job_peak_s = sum(2.0 * macs[KERNEL_LAYER[k]] * B / (kernel_peak(tr.engine.kernel_split(k)) * 1e12)
                     for k in dom_jobs) if dom_flops else None
    avg_ms = probe_ms / max(launches, 1)
    roof = None
    if dom_flops:
        split = tr.engine.kernel_split(dom)
        fam = tr.engine.kernel_family(dom)
        peak = dom_flops / job_peak_s / 1e12
        ach = dom_flops / (avg_ms / 1000.0) / 1e12
        if len(dom_jobs) > 1:
            path = "multi-job launch %s: %s" % ("+".join(dom_jobs), ", ".join(
                "%s %d products per fp32 product" % (k, tr.engine.kernel_split(k)) for k in dom_jobs))
        elif split <= 1:
            path = "fp32 MFMA"
        elif fam == 2:
            path = "fp16 MFMA, %d products per fp32 product (power-of-two scaled hi/lo split)" % split
        else:
            path = "bf16 MFMA, %d products per fp32 product (exact hi/mid/lo split)" % split
        roof = {"bound": "mfma", "kernel": dom, "jobs": dom_jobs, "achieved": round(ach, 2),
                "peak": round(peak, 1), "unit": "TFLOP/s", "frac": round(ach / peak, 4),
                "traffic": pmc_traffic(dom), "avg_launch_ms": round(avg_ms, 4),
                "launches": launches, "path": path,
                "peak_basis": "algorithmic fp32 FLOP/s: %s" % (
                    "fp32 MFMA 157.3 TF" if split <= 1 else
                    "2516.6 TF dense 16-bit MFMA / %d split products" % split if len(dom_jobs) == 1 else
                    "total FLOPs / sum over jobs of (job FLOPs / 2516.6 TF x its split products)")}
    step_tflops = train_step_flops(B, C, F, A) / (ms_step / 1000.0) / 1e12
    ceiling["step_frac_of_mixed_path_ceiling"] = round(ceiling["ideal_ms"] / ms_step, 4)

    out = {"metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 4),
           "ms_per_step_median": round(med_ms, 4),
           "value_median": round(world * B / (med_ms / 1000.0), 1),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "arith": ARITH,
           "data": "synthetic uint8 84x84x4 frames, random actions/returns, weights from the "
                   "reference initialisers (seed 0); resident in HBM",
           "config": {"workload": "configs[2]/[3]: BA3C train step (fwd+bwd+clip+%sAdam) "
                                  "B=%d/GPU, fc_neurons=%d, fc_splits=%d, A=%d"
                                  % ("RCCL mean+" if sync else "", B, F, S, A),
                      "global_batch": world * B, "per_gpu_batch": B, "fc_neurons": F,
                      "fc_splits": S, "num_actions": A, "parallelism": "dp%d" % world,
                      "step_path": "bucketed sync (phase-split backward, per-bucket clip, "
                                   "unfused update)" if sync else "fused single replica",
                      "backup_workers": 0},
           "step_tflops_algorithmic": round(step_tflops, 2),
           "ceiling": ceiling,
           "roofline": roof,
           "probe": {"kernel": dom, "avg_launch_ms": round(avg_ms, 4), "launches": launches,
                     "every": args.probe_every},
           "kernel_ms_per_step": {k: round(v, 4) for k, v in per_kernel.items()}}

    rc = health(out, flags, identical)
    if sync:
        ks = [int(k) for k in args.occupy.split(",") if k.strip()]
        out["exchange"] = exchange_report(tr, batch, max(args.steps // 3, 5), world, ks,
                                          args.occupy_us)
    if not args.no_overlap:
        out["overlap"] = overlap_bench(tr, batch, args.predict_batch, 10, world)
    if not args.no_b32:
        close_exchange(tr)
        del tr
        tr = None
        tr32, b32 = build_trainer(32, 128, 4, A, world, seed=rank, sync=sync)
        n32 = max(args.steps, 100)
        el32, med32, _, _ = time_steps(tr32, b32, n32, 10, world)
        out["b32"] = {"config": "configs[1]: B=32/GPU, fc_neurons=128, fc_splits=4",
                      "value": round(world * 32 * n32 / el32, 1), "unit": "samples/s",
                      "ms_per_step": round(el32 / n32 * 1000.0, 4),
                      "ms_per_step_median": round(med32, 4), "launch": "eager"}
        if world == 1 and not sync:
            elg = time_graph_steps(tr32, b32, n32, 10)
            out["b32"].update({"value_graph": round(32 * n32 / elg, 1),
                               "ms_per_step_graph": round(elg / n32 * 1000.0, 4)})
        f32 = tr32.engine.device_errors()
        if f32:
            out["b32"]["device_errors"] = int(f32)
            rc = 1
        tr = tr32
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(F, S, A, args.cpu_seconds)
        out["gpu_vs_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if sync:
        dist.barrier()
        close_exchange(tr)
        dist.destroy_process_group()
    return rc


def close_exchange(tr):
    """Destroy the trainer's direct RCCL communicator (before its process group goes)."""
    if tr is not None and hasattr(tr.optimizer, "close"):
        tr.optimizer.close()


if __name__ == "__main__":
    main()
