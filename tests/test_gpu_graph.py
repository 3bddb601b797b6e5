"""hipGraph-captured learner step (Ba3cTrainer.capture_step): replaying the captured
fwd+bwd+clip+Adam chain, with the inputs refilled in place between replays, reproduces the
eager step sequence bit for bit — Adam's bias-correction powers live on the device, so every
replay uses the step count's own alpha (TF's float32 beta-power variables)."""
import numpy as np
import pytest
import torch

from oracle import ba3c_oracle as O

pytestmark = pytest.mark.gpu


def _trainer(B):
    from ba3c_amd.model import Model
    from ba3c_amd.optimizer import AdamOptimizer
    from ba3c_amd.trainer import Ba3cTrainer, TrainConfig
    m = Model(num_actions=4, fc_neurons=128, fc_splits=4, batch_size=B, max_batch=B)
    m.engine.load_params(O.init_params(128, 4, 4, seed=5, dtype=np.float32))
    return Ba3cTrainer(TrainConfig(model=m, optimizer=AdamOptimizer(1e-3, 0.8, 0.75, 1e-8)))


def _batches(B, n):
    out = []
    for i in range(n):
        rs = np.random.RandomState(300 + i)
        out.append((torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda(),
                    torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda(),
                    torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()))
    return out


def test_captured_step_replays_match_eager_steps():
    B = 16
    bs = _batches(B, 4)
    eager = _trainer(B)
    for b in bs[1:]:                        # capture_step's warmup steps are undone
        eager.train_step(*b)
    torch.cuda.synchronize()

    cap = _trainer(B)
    static = tuple(t.clone() for t in bs[0])
    replay = cap.capture_step(*static, warmup=2)
    for b in bs[1:]:
        for dst, src in zip(static, b):
            dst.copy_(src)
        replay()
    torch.cuda.synchronize()
    assert cap.global_step == eager.global_step == 3
    np.testing.assert_array_equal(cap.engine.params.cpu().numpy(), eager.engine.params.cpu().numpy())
    b1, b2 = cap.optimizer.powers()
    e1, e2 = eager.optimizer.powers()
    assert (b1, b2) == (e1, e2)
    for s_cap, s_eag in zip(cap.optimizer.slots, eager.optimizer.slots):
        np.testing.assert_array_equal(s_cap.cpu().numpy(), s_eag.cpu().numpy())


@pytest.mark.parametrize("mode", ["side", "multi", "side_auto", "fused_update"])
def test_backward_launch_paths_match_single_stream(monkeypatch, mode):
    """At B <= 128 the backward runs either as multi-job launches (default: each layer's input-
    and weight-gradient kernels in one grid, ba3c_multi.h) or with the weight gradients on a
    second HIP stream (BA3C_MULTI=0, or BA3C_OVERLAP=1: fork/join events); the fused-clip Adam
    apply is one grid-barrier launch (clip_update_kernel) unless BA3C_FUSED_UPDATE=0.  Eager and
    graph-captured steps of every variant must equal the plainest path (one stream, one kernel
    per product, sumsq + update launches) bit for bit, TfDictOp scalars included."""
    B = 64
    bs = _batches(B, 4)
    plain = {"BA3C_OVERLAP": "0", "BA3C_MULTI": "0", "BA3C_FUSED_UPDATE": "0"}
    variant = {"side": {"BA3C_OVERLAP": "1"},
               "multi": {},
               "side_auto": {"BA3C_MULTI": "0"},
               "fused_update": {"BA3C_OVERLAP": "0", "BA3C_MULTI": "0"}}[mode]
    for k, v in plain.items():
        monkeypatch.setenv(k, v)
    ref = _trainer(B)
    for b in bs[1:]:
        ref.train_step(*b)
    ref_scalars = ref.model.scalars_dict()
    for k in plain:
        monkeypatch.delenv(k)
    for k, v in variant.items():
        monkeypatch.setenv(k, v)
    eager = _trainer(B)
    for b in bs[1:]:
        eager.train_step(*b)
    assert eager.model.scalars_dict() == ref_scalars
    cap = _trainer(B)
    static = tuple(t.clone() for t in bs[0])
    replay = cap.capture_step(*static, warmup=2)
    for b in bs[1:]:
        for dst, src in zip(static, b):
            dst.copy_(src)
        replay()
    torch.cuda.synchronize()
    want = ref.engine.params.cpu().numpy()
    np.testing.assert_array_equal(eager.engine.params.cpu().numpy(), want)
    np.testing.assert_array_equal(cap.engine.params.cpu().numpy(), want)
    for s_cap, s_ref in zip(cap.optimizer.slots, ref.optimizer.slots):
        np.testing.assert_array_equal(s_cap.cpu().numpy(), s_ref.cpu().numpy())
    assert cap.optimizer.powers() == ref.optimizer.powers()
    for tr in (ref, eager, cap):
        assert tr.engine.device_errors() == 0      # no in-launch wait gave up


def test_large_batch_fc1_multi_job_matches_separate_launches(monkeypatch):
    """Above OVERLAP_B the fc1 input gradient and the head / fc1 weight gradients run as one
    multi-job launch (default) or as three launches (BA3C_MULTI_BIG=0): same gradients and
    scalars bit for bit (B=160, F=512, S=1: the bench geometry)."""
    from ba3c_amd.engine import Ba3cEngine
    B = 160
    rs = np.random.RandomState(77)
    state = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda()
    action = torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda()
    R = torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()
    params = O.init_params(512, 1, 4, seed=7, dtype=np.float32)
    out = []
    for env in ("0", None):
        if env is None:
            monkeypatch.delenv("BA3C_MULTI_BIG", raising=False)
        else:
            monkeypatch.setenv("BA3C_MULTI_BIG", env)
        eng = Ba3cEngine(num_actions=4, fc_neurons=512, fc_splits=1, max_batch=B)
        eng.load_params(params)
        sc = eng.train_grads(state, action, R)
        torch.cuda.synchronize()
        out.append((eng.grads.clone(), sc.clone()))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


def test_ring_walk_band_kernels_match_one_band_kernels(monkeypatch):
    """From B = 2 x CUs up, conv1's forward and input gradient run as ring-walk persistent
    kernels (whole images per workgroup, halo rows carried in LDS) instead of one band per
    workgroup (BA3C_RING=0): activations, dp0, gradients and scalars bit for bit equal (conv1's
    input gradient dense on both sides: BA3C_C1D_SPARSE=0)."""
    from ba3c_amd.engine import Ba3cEngine
    monkeypatch.setenv("BA3C_C1D_SPARSE", "0")
    B = 2 * torch.cuda.get_device_properties(0).multi_processor_count
    rs = np.random.RandomState(78)
    state = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda()
    action = torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda()
    R = torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()
    params = O.init_params(512, 1, 4, seed=8, dtype=np.float32)
    out = []
    for env in ("0", None):
        if env is None:
            monkeypatch.delenv("BA3C_RING", raising=False)
        else:
            monkeypatch.setenv("BA3C_RING", env)
        eng = Ba3cEngine(num_actions=4, fc_neurons=512, fc_splits=1, max_batch=B)
        eng.load_params(params)
        sc = eng.train_grads(state, action, R)
        ws = {n: eng.workspace_tensor(n, B).clone() for n in ("p1", "c1", "dp0")}
        torch.cuda.synchronize()
        out.append((eng.grads.clone(), sc.clone(), ws))
    assert torch.equal(out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])
    for n in out[0][2]:
        assert torch.equal(out[0][2][n], out[1][2][n]), n


def test_ring_walk_dynamic_image_queue_matches_static_ranges(monkeypatch):
    """At the bench's B=2048 (8 x CUs: four images per ring-walk workgroup) conv1's forward and
    input gradient draw their images from a dynamic queue (one agent-scope ticket per image,
    BA3C_DYNQ=1) instead of static contiguous ranges (BA3C_DYNQ=0, the default): activations,
    argmax codes, dp0, every gradient and the scalars bit for bit equal, over two steps (the
    tickets are re-zeroed by each step's weight-prep launch), and the predictor forward too."""
    from ba3c_amd.engine import Ba3cEngine
    B = 8 * torch.cuda.get_device_properties(0).multi_processor_count
    rs = np.random.RandomState(91)
    state = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda()
    action = torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda()
    R = torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()
    params = O.init_params(512, 1, 4, seed=21, dtype=np.float32)
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv("BA3C_DYNQ", env)
        eng = Ba3cEngine(num_actions=4, fc_neurons=512, fc_splits=1, max_batch=B)
        eng.load_params(params)
        got = []
        for _ in range(2):
            sc = eng.train_grads(state, action, R)
            got.append(eng.grads.clone())
            got.append(sc.clone())
        got += [eng.workspace_tensor(n, B).clone() for n in ("p1", "c1", "dp0", "dp1")]
        got += [t.clone() for t in eng.forward(state)]
        torch.cuda.synchronize()
        assert eng.device_errors() == 0
        out.append(got)
        del eng
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


def _dp0_float64(dp1, c1, w1, B):
    """conv1's input gradient in float64 from the GPU's pooled gradient dP1 [B,18,18,32], its
    argmax codes (255: ReLU / pool gradient 0) and conv1/W (HWIO): dZ1 un-pooled to 36x36, then
    the transposed VALID convolution onto p0's 40x40.  Returns (dP0 NHWC, the same with |dZ1|
    and |W1|: the sum of the magnitudes of every element's terms)."""
    import torch.nn.functional as Fn
    d = dp1.double().cpu().reshape(B, 18, 18, 32)
    c = c1.cpu().reshape(B, 18, 18, 32).to(torch.int64)
    dz = torch.zeros(B, 36, 36, 32, dtype=torch.float64)
    for pos in range(4):
        dz[:, pos // 2::2, pos % 2::2, :] = torch.where(c == pos, d, torch.zeros_like(d))
    dz = dz.permute(0, 3, 1, 2)
    w = torch.tensor(np.asarray(w1, np.float64)).permute(3, 2, 0, 1)     # OIHW
    ex = Fn.conv_transpose2d(dz, w).permute(0, 2, 3, 1).numpy()
    mg = Fn.conv_transpose2d(dz.abs(), w.abs()).permute(0, 2, 3, 1).numpy()
    return ex, mg


@pytest.mark.parametrize("frames", ["random", "atari"])
def test_sparse_conv1_input_gradient_matches_dense(monkeypatch, frames):
    """conv1's input gradient on 2:4-sparse MFMA (ba3c_dgrad1s.h, BA3C_C1D_SPARSE=1, used from
    B = 2 x CUs; off by default: slower) against the dense ring walk (BA3C_C1D_SPARSE=0, the
    default) on the same inputs: the same products minus
    exact zeros, summed in another order — dP0 within its error-model bound (normwise, per
    image; both are fp32-class, ~1e-6 apart), conv0/W's gradient (the only tensor dP0 feeds) within 1e-5, every other gradient,
    the scalars, p1 and the codes bit for bit.  dP0 of each side is held element by element to
    its error-model bound against a float64 evaluation from the same inputs (_dp0_float64)."""
    from atari_frames import atari_frames
    from ba3c_amd.engine import Ba3cEngine
    B = 2 * torch.cuda.get_device_properties(0).multi_processor_count
    rs = np.random.RandomState(81)
    if frames == "random":
        state = rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)
        params = O.init_params(512, 1, 4, seed=8, dtype=np.float32)
    else:
        state = atari_frames(B, 81)
        params = {k: (v * np.float32(2.0)).astype(np.float32)
                  for k, v in O.init_params(512, 1, 4, seed=8, dtype=np.float32).items()}
    state = torch.from_numpy(state).cuda()
    action = torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda()
    R = torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()
    out = []
    for env in ("0", "1"):
        monkeypatch.setenv("BA3C_C1D_SPARSE", env)
        eng = Ba3cEngine(num_actions=4, fc_neurons=512, fc_splits=1, max_batch=B)
        eng.load_params(params)
        sc = eng.train_grads(state, action, R)
        ws = {n: eng.workspace_tensor(n, B).clone() for n in ("p1", "c1", "dp0", "dp1")}
        g = {k: v.copy() for k, v in eng.state_dict(eng.grads).items()}
        torch.cuda.synchronize()
        out.append((g, sc.clone(), ws))
        assert eng.device_errors() == 0
        del eng
    (gd, sd, wd), (gs, ss, wsp) = out
    assert torch.equal(sd, ss)
    assert torch.equal(wd["p1"], wsp["p1"]) and torch.equal(wd["c1"], wsp["c1"])
    # error model (Higham's gamma_n): each side evaluates every dP0 element
    # as K = 800 split products (hi*hi + hi*lo + lo*hi, <= 3 x 2^-22 relative each) accumulated
    # in fp32 (n = 3 x 800 roundings), so |computed - exact| <= (gamma_n + 3 x 2^-22) x
    # sum_k |dZ1_k W1_k| per element, the exact value and the sum of magnitudes evaluated here
    # in float64 from the same dP1 / codes / W1 (bound fixed before the run; the normwise
    # difference of the two orders is reported beside it)
    exact, mag = _dp0_float64(wd["dp1"], wd["c1"], params["conv1/W"], B)
    n, u = 3 * 800, 2.0 ** -24
    # + elements below 2^-17 of their image's (tensor's) max keep an absolute accuracy of
    # 2^-39 x that max in fp16 hi + lo: over 800 terms of both operands <= 2^-28 x M x Wmax
    m_img = wd["dp1"].double().abs().reshape(B, -1).max(dim=1).values.cpu().numpy()
    wmax = float(np.abs(params["conv1/W"]).max())
    bound = (n * u / (1 - n * u) + 3 * 2.0 ** -22) * mag + \
        2.0 ** -28 * m_img.reshape(B, 1, 1, 1) * wmax
    for name, side in (("dense", wd["dp0"]), ("sparse", wsp["dp0"])):
        got = side.double().cpu().numpy().reshape(exact.shape)
        ratio = (np.abs(got - exact) / np.maximum(bound, 1e-300)).max()
        print("dp0 %s: max |err| / model bound %.3f" % (name, ratio))
        assert np.all(np.abs(got - exact) <= bound), name
    d = wd["dp0"].double().reshape(B, -1).cpu().numpy()
    e = wsp["dp0"].double().reshape(B, -1).cpu().numpy()
    err = np.abs(e - d).max(axis=1) / np.maximum(np.abs(d).max(axis=1), 1e-30)
    print("dp0 sparse vs dense, per-image normwise: max %.2e" % err.max())
    for k in gd:
        if k == "conv0/W":
            r = np.abs(gs[k] - gd[k]).max() / np.abs(gd[k]).max()
            print("conv0/W rel err %.2e" % r)
            assert r < 1e-5, r
        else:
            assert np.array_equal(gs[k], gd[k]), k


@pytest.mark.parametrize("B", [32, 160])
def test_two_phase_backward_equals_one_pass(B):
    """ba3c_train_grads_phase 1 then 2 (the bucketed data-parallel step splits the pass at the
    fc1 + heads bucket) gives the one-pass gradients and scalars bit for bit; after phase 1 the
    bucket's tensors are already final."""
    from ba3c_amd.engine import Ba3cEngine
    rs = np.random.RandomState(79)
    state = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda()
    action = torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda()
    R = torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()
    eng = Ba3cEngine(num_actions=4, fc_neurons=128, fc_splits=4, max_batch=B)
    eng.load_params(O.init_params(128, 4, 4, seed=9, dtype=np.float32))
    sc = eng.train_grads(state, action, R).clone()
    ref = eng.grads.clone()
    eng.grads.fill_(0.5)                       # every tensor element must be rewritten
    eng.train_grads(state, action, R, phase=1)
    t, off = eng.bucket_split()
    assert eng.layout[t][0].startswith("fc1")
    mid = eng.grads.clone()
    # The overlap contract of the bucketed exchange (trainer.py _bucketed_sync_step): while
    # the bucket [off:] is being all-reduced, phase 2 must not write it at all — a sentinel
    # there survives phase 2 — and must rewrite every conv gradient element [:off].
    eng.grads[off:] = 7.25
    eng.grads[:off] = -3.5
    sc1 = eng.train_grads(state, action, R, phase=2)
    torch.cuda.synchronize()
    assert bool((eng.grads[off:] == 7.25).all())
    for i, (name, o, n, _) in enumerate(eng.layout):   # (the 64-float alignment gaps are not
        if i >= t:                                      # gradient elements)
            assert torch.equal(mid[o:o + n], ref[o:o + n]), name
        else:
            assert torch.equal(eng.grads[o:o + n], ref[o:o + n]), name
    assert torch.equal(sc1, sc)


@pytest.mark.parametrize("B", [32, 2048])
def test_held_phase1_reduction_on_exchange_stream_equals_one_pass(B):
    """The N>1 step's order (trainer.py _bucketed_sync_step): phase 4 (phase 1 with the fc1 +
    heads reduction held), phase 2 recording the handle's phase-2 event after conv3, then on a
    second stream that waits for the event the held reduction (ba3c_launch_held) and the
    bucket's clip in its two-launch form (ba3c_clip_grads_range2 BA3C_CLIP_NO_RESIDENCY).
    Gradients equal the one-pass gradients bit for bit (B=2048: the bench's persistent
    kernels), the clipped bucket equals the one-launch clip of the same gradients, phase 2
    leaves the bucket alone, and no in-launch wait gave up."""
    from ba3c_amd import hipevent
    from ba3c_amd.engine import Ba3cEngine
    F, S = (128, 4) if B == 32 else (512, 1)
    rs = np.random.RandomState(83)
    state = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda()
    action = torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda()
    R = torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()
    eng = Ba3cEngine(num_actions=4, fc_neurons=F, fc_splits=S, max_batch=B)
    eng.load_params(O.init_params(F, S, 4, seed=13, dtype=np.float32))
    tb, off = eng.bucket_split()
    nt = len(eng.layout)
    sc = eng.train_grads(state, action, R).clone()
    ref = eng.grads.clone()
    eng.clip_grads_range(tb, nt)                 # one-launch clip of the bucket
    ref_clip = eng.grads[off:].clone()
    mid = hipevent.HipEvent(hipevent.HIP_EVENT_DISABLE_TIMING | hipevent.HIP_EVENT_RELEASE_TO_DEVICE)
    eng.set_phase2_event(mid)
    side = torch.cuda.Stream()
    for _ in range(2):                           # a second step on the same handle
        eng.grads.fill_(0.5)
        eng.train_grads(state, action, R, phase=4)
        sc2 = eng.train_grads(state, action, R, phase=2)
        mid.wait(side)
        eng.launch_held(side)
        hipevent.wait_stream(torch.cuda.current_stream(), side)
        torch.cuda.synchronize()
        for i, (name, o, n, _) in enumerate(eng.layout):
            assert torch.equal(eng.grads[o:o + n], ref[o:o + n]), name
        assert torch.equal(sc2, sc)
        with torch.cuda.stream(side):
            eng.clip_grads_range(tb, nt, no_residency=True)
        torch.cuda.synchronize()
        _bucket_equal(eng, tb, off, ref_clip)
    eng.set_phase2_event(None)
    # an unlaunched held reduction is launched by the next entry point on its own stream
    eng.train_grads(state, action, R, phase=4)
    eng.train_grads(state, action, R, phase=2)
    eng.clip_grads_range(tb, nt, no_residency=True)
    torch.cuda.synchronize()
    _bucket_equal(eng, tb, off, ref_clip)
    assert eng.device_errors() == 0


def _bucket_equal(eng, tb, off, ref_clip):
    for i, (name, o, n, _) in enumerate(eng.layout):     # tensors only (not the alignment gaps)
        if i >= tb:
            assert torch.equal(eng.grads[o:o + n], ref_clip[o - off:o - off + n]), name


def test_one_launch_bucket_clip_matches_two_launch_clip(monkeypatch):
    """ba3c_clip_grads_range (the data-parallel step's per-bucket clip, train.py:329-330 per
    replica) runs as ONE launch with tagged partials (clip_range_kernel); BA3C_FUSED_UPDATE=0
    keeps sumsq + clip launches.  Same gradients in, bit-identical clipped buckets out, over
    repeated calls on both buckets (the tags advance per chunk), and no wait gave up."""
    from ba3c_amd.engine import Ba3cEngine
    B = 32
    rs = np.random.RandomState(41)
    state = torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda()
    action = torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda()
    R = torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()
    params = O.init_params(512, 1, 4, seed=8, dtype=np.float32)
    out = []
    for fused in ("1", "0"):
        monkeypatch.setenv("BA3C_FUSED_UPDATE", fused)
        eng = Ba3cEngine(num_actions=4, fc_neurons=512, fc_splits=1, max_batch=B)
        eng.load_params(params)
        tb, _ = eng.bucket_split()
        nt = len(eng.layout)
        got = []
        for step in range(3):
            eng.train_grads(state, action, R)
            eng.clip_grads_range(tb, nt)
            eng.clip_grads_range(0, tb)
            got.append(eng.grads.clone())
            eng.grads.mul_(1.5 + step)                   # a second clip of other values
            eng.clip_grads_range(0, tb)
            got.append(eng.grads.clone())
        torch.cuda.synchronize()
        assert eng.device_errors() == 0
        out.append(got)
        del eng
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [32, 48])
def test_chained_launches_match_separate_launches(monkeypatch, B):
    """Chained multi-job launch (ba3c_multi.h launch_chain, default at B <= 51; BA3C_CHAIN=0:
    two launches): the zeroing of the ReLU counters / max slots signals inside the launch, and
    conv0's forward splits its own weight fragments and waits for it only before publishing.
    Outputs must be bit-identical: training gradients and scalars over repeated steps (the
    counter words reset at every launch's end), the predictor's probabilities and values, graph
    replays at B=32; no wait gave up."""
    from ba3c_amd.engine import Ba3cEngine
    rs = np.random.RandomState(B)
    batches = []
    for _ in range(3):
        batches.append((torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda(),
                        torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda(),
                        torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()))
    params = O.init_params(128, 4, 4, seed=9, dtype=np.float32)
    out = []
    for env in ("0", None):
        if env is None:
            monkeypatch.delenv("BA3C_CHAIN", raising=False)
        else:
            monkeypatch.setenv("BA3C_CHAIN", env)
        eng = Ba3cEngine(num_actions=4, fc_neurons=128, fc_splits=4, max_batch=B)
        eng.load_params(params)
        got = []
        for state, action, R in batches:
            sc = eng.train_grads(state, action, R)
            got += [eng.grads.clone(), sc.clone()]
            probs, probsT, value = eng.forward(state)
            got += [probs.clone(), probsT.clone(), value.clone()]
        torch.cuda.synchronize()
        assert eng.device_errors() == 0
        out.append(got)
        del eng
    for a, b in zip(out[0], out[1]):
        assert torch.equal(a, b)
    if B == 32:
        monkeypatch.setenv("BA3C_CHAIN", "0")
        plain = _trainer(B)
        monkeypatch.delenv("BA3C_CHAIN")
        cap = _trainer(B)
        bs = _batches(B, 4)
        for b in bs[1:]:
            plain.train_step(*b)
        static = tuple(t.clone() for t in bs[0])
        replay = cap.capture_step(*static, warmup=2)
        for b in bs[1:]:
            for dst, src in zip(static, b):
                dst.copy_(src)
            replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(cap.engine.params.cpu().numpy(), plain.engine.params.cpu().numpy())
        assert cap.engine.device_errors() == 0


@pytest.mark.parametrize("B,opt", [(32, "adam"), (32, "rms"), (160, "gd")])
def test_deferred_reduction_rides_on_fused_apply(B, opt):
    """ba3c_train_grads_phase(phase 3) leaves the pass's weight-gradient reduction pending and
    the next fused-clip apply runs it as the signalling job of ONE chained launch (reduce ->
    clip + update).  Against phase 0 + the same apply: the same raw gradients and bit-identical
    parameters and slots over repeated steps (host and device Adam powers), the reduction
    reported as merged into the update launch, and no wait gave up.  A phase-3 pass followed
    by any other call (forward, unfused clip — also on another stream) first launches the
    pending reduction itself."""
    from ba3c_amd.engine import Ba3cEngine
    from ba3c_amd.optimizer import AdamOptimizer, GradientDescentOptimizer, RMSPropOptimizer
    mk = {"adam": lambda: AdamOptimizer(1e-3, 0.8, 0.75, 1e-8), "rms": lambda: RMSPropOptimizer(1e-3),
          "gd": lambda: GradientDescentOptimizer(1e-2)}[opt]
    rs = np.random.RandomState(B + 7)
    batches = [(torch.from_numpy(rs.randint(0, 256, size=(B, 84, 84, 4)).astype(np.uint8)).cuda(),
                torch.from_numpy(rs.randint(0, 4, size=B).astype(np.int64)).cuda(),
                torch.from_numpy(rs.normal(size=B).astype(np.float32)).cuda()) for _ in range(3)]
    params = O.init_params(128, 4, 4, seed=11, dtype=np.float32)
    out = []
    for phase in (0, 3):
        eng = Ba3cEngine(num_actions=4, fc_neurons=128, fc_splits=4, max_batch=B)
        eng.load_params(params)
        o = mk()
        if opt == "adam":
            o.use_device_state(eng.device)
        got = []
        for state, action, R in batches:
            sc = eng.train_grads(state, action, R, phase=phase)
            o.apply_gradients(eng, fuse_clip=True)
            got += [sc.clone(), eng.grads.clone(), eng.params.clone()] + [s.clone() for s in o.slots]
            merged = eng.kernel_merged("update")
            assert ("wgrad_reduce" in merged) == (phase == 3), merged
        # phase 3, then calls that are not a fused apply: the pending reduction runs first
        eng.train_grads(*batches[0], phase=phase)
        eng.forward(batches[1][0])
        got.append(eng.grads.clone())
        eng.train_grads(*batches[1], phase=phase)
        eng.clip_grads()
        got.append(eng.grads.clone())
        # a call on another stream ordered after the pass by the caller's own event (recorded
        # before the pending reduction was launched) still sees the reduced gradient
        eng.train_grads(*batches[2], phase=phase)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            eng.clip_grads()
        torch.cuda.current_stream().wait_stream(side)
        got.append(eng.grads.clone())
        torch.cuda.synchronize()
        assert eng.device_errors() == 0
        out.append(got)
        del eng
    assert len(out[0]) == len(out[1])
    for i, (a, b) in enumerate(zip(out[0], out[1])):
        assert torch.equal(a, b), i
