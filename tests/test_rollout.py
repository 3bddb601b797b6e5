"""Learner input side: n-step returns, batch assembly and frame
history on the GPU against the reference's own simulator-master logic restated in the oracle
(train.py:364-437, RL/simulator.py:160-185, RL/history.py:12-55).  Integer / index work is
bit-exact; R is the float32 cast of the float64 recursion, compared bit for bit."""
import numpy as np
import pytest
import torch

from oracle import ba3c_oracle as O


# ---- oracle pinning (CPU) -------------------------------------------------------------------
def test_parse_memory_hand_example():
    """6 transitions, not over: the newest only bootstraps; R runs backwards with clip."""
    mem = [{"reward": r, "id": i} for i, r in enumerate([0.0, 3.0, -0.5, 1.0, -7.0, 9.0])]
    dps, left = O.parse_memory(mem, np.float32(0.25), False)
    assert [d[0]["id"] for d in dps] == [4, 3, 2, 1, 0] and left[0]["id"] == 5
    R = 0.25
    want = []
    for r in [-7.0, 1.0, -0.5, 3.0, 0.0]:
        R = max(-1.0, min(1.0, r)) + 0.99 * R
        want.append(R)
    np.testing.assert_array_equal([d[1] for d in dps], want)
    dps, left = O.parse_memory(mem[:3], 0, True)
    assert [d[0]["id"] for d in dps] == [2, 1, 0] and left == []
    assert dps[0][1] == -0.5


def test_history_state_pads_with_zeros():
    f = [np.full((2, 2, 1), v, np.uint8) for v in (7, 8)]
    s = O.history_state(f, 4)
    assert s.shape == (2, 2, 4) and list(s[0, 0]) == [0, 0, 7, 8]
    s = O.history_state(f + [f[0] + 2, f[0] + 3, f[0] + 4], 4)
    assert list(s[1, 1]) == [8, 9, 10, 11]


# ---- GPU ------------------------------------------------------------------------------------
def _encode(E, t, C=4):
    """States whose first two pixels carry (env, step) as little-endian int32."""
    st = np.zeros((E, 84, 84, C), np.uint8)
    for e in range(E):
        st[e, 0, 0, :4] = np.frombuffer(np.int32(e).tobytes(), np.uint8)
        st[e, 0, 1, :4] = np.frombuffer(np.int32(t).tobytes(), np.uint8)
    return st


def _decode(st):
    b = np.ascontiguousarray(st[:, 0, :2, :4]).reshape(-1, 8)
    return [(int(np.frombuffer(x[:4].tobytes(), np.int32)[0]), int(np.frombuffer(x[4:].tobytes(), np.int32)[0]))
            for x in b]


@pytest.mark.gpu
@pytest.mark.parametrize("E,steps,p_over", [(37, 40, 0.08), (1, 25, 0.0), (300, 13, 0.3)])
def test_nstep_returns_match_simulator_master(E, steps, p_over):
    from ba3c_amd.rollout import BatchQueue, RolloutBuffer
    rs = np.random.RandomState(E)
    buf = RolloutBuffer(E, channels=4)
    mirror = O.SimulatorMasterMirror()
    got, want = [], []
    q = BatchQueue(16)
    batches = []
    for t in range(steps):
        if t > 0:
            rew = rs.choice([0.0, 1.0, -1.0, 2.0, -3.0, 0.5, 30.0], size=E).astype(np.float64)
            over = rs.rand(E) < p_over
            for e in range(E):
                mirror.on_message(e, float(rew[e]), bool(over[e]))
            dps = buf.on_reward(torch.from_numpy(rew), torch.from_numpy(over))
            q.put(dps)
            while True:
                b = q.get()
                if b is None:
                    break
                batches.append([x.cpu().numpy() for x in b])
            got.extend(zip(_decode(dps.state.cpu().numpy()), dps.action.cpu().numpy().tolist(),
                           dps.R.cpu().numpy().tolist(), dps.init_R.cpu().numpy().tolist(),
                           dps.over.cpu().numpy().tolist()))
        act = rs.randint(0, 4, size=E).astype(np.int64)
        val = rs.normal(size=E).astype(np.float32)
        st = _encode(E, t)
        for e in range(E):
            mirror.on_state(e, (e, t), int(act[e]), val[e])
        buf.on_state(torch.from_numpy(st).cuda(), torch.from_numpy(act).cuda(),
                     torch.from_numpy(val).cuda())
    for k, R, init_r, over in mirror.queue:
        want.append((k["state"], k["action"], float(np.float32(R)), float(np.float32(init_r)), int(over)))
    assert len(got) == len(want) and len(want) > 0
    for g, w in zip(got, want):
        assert g == w, (g, w)
    # BatchData(16): consecutive, in order
    flat = [dp for b in batches for dp in _decode(b[0])]
    assert flat == [w[0] for w in want[:len(flat)]] and len(flat) == 16 * len(batches)


@pytest.mark.gpu
def test_history_push_matches_history_frame_player():
    from ba3c_amd.rollout import FrameHistory
    E, steps = 9, 14
    rs = np.random.RandomState(3)
    hist = FrameHistory(E, hist_len=4, channels=1)
    frames_seen = [[] for _ in range(E)]
    for t in range(steps):
        fr = rs.randint(0, 256, size=(E, 84, 84, 1)).astype(np.uint8)
        over = rs.rand(E) < 0.2 if t > 0 else np.zeros(E, bool)
        state = hist.push(torch.from_numpy(fr).cuda(), torch.from_numpy(over).cuda()).cpu().numpy()
        for e in range(E):
            if over[e]:
                frames_seen[e] = []
            frames_seen[e].append(fr[e])
            np.testing.assert_array_equal(state[e], O.history_state(frames_seen[e], 4))


@pytest.mark.gpu
def test_history_push_generic_channels():
    """RGB frames (c=3, C=12: the reference's own pipeline, train.py:116-119)."""
    from ba3c_amd.rollout import FrameHistory
    E = 3
    rs = np.random.RandomState(4)
    hist = FrameHistory(E, hist_len=4, channels=3)
    seen = [[] for _ in range(E)]
    for t in range(6):
        fr = rs.randint(0, 256, size=(E, 84, 84, 3)).astype(np.uint8)
        over = np.array([False, t == 3, False])
        state = hist.push(torch.from_numpy(fr).cuda(), torch.from_numpy(over).cuda()).cpu().numpy()
        for e in range(E):
            if over[e]:
                seen[e] = []
            seen[e].append(fr[e])
            np.testing.assert_array_equal(state[e], O.history_state(seen[e], 4))
