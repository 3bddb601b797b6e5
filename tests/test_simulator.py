"""Simulator side on CPU: the players / wrappers of RL/envbase.py,
RL/history.py and RL/common.py, the msgpack wire format of utils/serialize.py, and the
c2s / s2c protocol of RL/simulator.py between real simulator processes and the master, whose
datapoints are checked against the oracle's restatement of the master's memory logic
(oracle.SimulatorMasterMirror, train.py:364-437) replayed on the same message log."""
import os
import tempfile
import time

import numpy as np
import pytest

from ba3c_amd import envs, simulator as S
from oracle import ba3c_oracle as O


def test_serialize_round_trip():
    st = np.arange(84 * 84 * 4, dtype=np.uint8).reshape(84, 84, 4)
    msg = (b"simulator-3", st, 1.5, True, 7, True)
    back = S.loads(S.dumps(msg))
    assert back[0] == b"simulator-3" and back[2:] == [1.5, True, 7, True]
    assert back[1].dtype == np.uint8 and back[1].shape == st.shape and (back[1] == st).all()
    a, ts, alive = S.loads(S.dumps((np.int64(3), 12, False)))
    assert int(a) == 3 and ts == 12 and alive is False
    f = np.linspace(-1, 1, 7).astype(np.float32)
    assert (S.loads(S.dumps(f)) == f).all()


def test_history_frame_player_matches_reference_concat():
    pl = envs.HistoryFramePlayer(envs.SyntheticAtariPlayer(idx=2, seed=5), 4)
    frames = [pl.player.current_state()[:, :, None]]
    for t in range(150):
        st = pl.current_state()
        assert st.shape == (84, 84, 4) and st.dtype == np.uint8
        np.testing.assert_array_equal(st, O.history_state(frames, 4))
        r, over = pl.action(t % 4)
        f = pl.player.current_state()[:, :, None]
        frames = [f] if over else frames + [f]


def test_prevent_stuck_and_limit_length():
    class Rec(envs.RLEnvironment):
        def __init__(self):
            super(Rec, self).__init__()
            self.acts, self.restarts, self.finished = [], 0, 0

        def current_state(self):
            return np.zeros((84, 84), np.uint8)

        def action(self, act):
            self.acts.append(act)
            return 0.0, False

        def restart_episode(self):
            self.restarts += 1

        def finish_episode(self):
            self.finished += 1

    rec = Rec()
    pl = envs.PreventStuckPlayer(rec, 30, 1)
    for _ in range(29):
        pl.action(0)
    assert rec.acts == [0] * 29
    pl.action(0)                      # the 30th identical action is replaced by FIRE (1)
    assert rec.acts[-1] == 1
    pl.action(0)
    assert rec.acts[-1] == 1          # the window still holds 30 zeros
    pl.action(2)
    assert rec.acts[-1] == 2

    rec2 = Rec()
    lim = envs.LimitLengthPlayer(rec2, 5)
    overs = [lim.action(0)[1] for _ in range(12)]
    assert overs == [False] * 4 + [True] + [False] * 4 + [True] + [False] * 2
    assert rec2.finished == 2 and rec2.restarts == 2

    rec3 = Rec()
    rec3.action = lambda act: (1.0, True)
    ar = envs.AutoRestartPlayer(rec3)
    assert ar.action(0) == (1.0, True) and rec3.finished == 1 and rec3.restarts == 1


def test_synthetic_player_episode_and_stats():
    pl = envs.get_player(idx=1, seed=3, train=False)
    space = pl.get_action_space()
    assert space.num_actions() == 4
    score = pl.play_one_episode(lambda s: 0)
    assert len(score) == 0 or isinstance(score, list)


class LoggingMaster(S.FunctionSimulatorMaster):
    """Records every handled message and decision for the oracle replay."""

    def __init__(self, *a, **kw):
        super(LoggingMaster, self).__init__(*a, **kw)
        self.log = []

    def handle(self, msg):
        ident, state, reward, is_over, ts, alive = msg
        if alive and not self._stop_req.is_set():
            self.log.append(("msg", ident, float(reward), bool(is_over)))
        return super(LoggingMaster, self).handle(msg)

    def _on_state(self, state, ident):
        n0 = len(self.clients[ident[0]].memory)
        super(LoggingMaster, self)._on_state(state, ident)
        t = self.clients[ident[0]].memory[-1]
        assert len(self.clients[ident[0]].memory) == n0 + 1
        self.log.append(("state", ident[0], int(state.sum()), t.action, float(t.value)))


def test_simulator_processes_and_master_protocol():
    d = tempfile.mkdtemp(prefix="ba3c_ipc_")
    c2s, s2c = "ipc://" + os.path.join(d, "c2s"), "ipc://" + os.path.join(d, "s2c")
    n = 3

    def policy(state):
        v = float(state[:, :, -1].mean()) / 255.0
        p = np.array([0.1, 0.2, 0.3, 0.4]) if int(state.sum()) % 2 else np.full(4, 0.25)
        return p, v

    master = LoggingMaster(c2s, s2c, n, policy, rs=np.random.RandomState(11))
    procs = S.start_simulators(S.SyntheticSimulatorWorker, n, c2s, s2c, seed=100)
    master.start()
    t0 = time.time()
    while len(master.queue) < 300 and time.time() - t0 < 60:
        time.sleep(0.02)
    master.stop()
    master.join(timeout=30)
    for p in procs:
        p.join(timeout=30)
    master.close()
    assert not master.is_alive() and master.is_done
    assert all(p.exitcode == 0 for p in procs)
    assert len(master.queue) >= 300

    # replay the log through the oracle's restatement of the master's memory logic
    mirror = O.SimulatorMasterMirror()
    for e in master.log:
        if e[0] == "msg":
            mirror.on_message(e[1], e[2], e[3])
        else:
            mirror.on_state(e[1], e[2], e[3], e[4])
    got = master.queue[:len(mirror.queue)]
    assert len(mirror.queue) == len(master.queue)
    for (st, act, R, ts, init_r, over), (tr, R_ref, init_ref, over_ref) in zip(got, mirror.queue):
        assert int(st.sum()) == tr["state"] and act == tr["action"]
        assert R == R_ref and float(init_r) == float(init_ref) and over == over_ref
    # every simulator contributed datapoints, episodes ended and n-step parses happened
    assert len({e[1] for e in master.log if e[0] == "msg"}) == n
    assert any(dp[5] for dp in master.queue) and any(not dp[5] for dp in master.queue)


def test_batched_master_rounds_match_per_message_memory_logic():
    """BatchedSimulatorMaster (one batch_policy call per round) over real simulator processes:
    its datapoints equal the oracle's restatement of the per-message master replayed on the
    same message log and decisions, and the actions are np.random.choice draws of one
    RandomState in arrival order."""
    from ba3c_amd.simulator_gpu import BatchedSimulatorMaster

    d = tempfile.mkdtemp(prefix="ba3c_ipcb_")
    c2s, s2c = "ipc://" + os.path.join(d, "c2s"), "ipc://" + os.path.join(d, "s2c")
    n = 4
    rs = np.random.RandomState(21)
    log = []

    def batch_policy(states):
        probs = np.array([[0.1, 0.2, 0.3, 0.4] if int(s.sum()) % 2 else [0.25] * 4 for s in states])
        values = np.array([float(s[:, :, -1].mean()) / 255.0 for s in states])
        actions = np.array([rs.choice(4, p=p) for p in probs])
        log.append(("round", [int(s.sum()) for s in states], actions.tolist(), values.tolist()))
        return probs, values, actions

    class Master(BatchedSimulatorMaster):
        def handle(self, msg):
            ident, state, reward, is_over, ts, alive = msg
            if alive and not self._stop_req.is_set():
                log.append(("msg", ident, float(reward), bool(is_over)))
            return super(Master, self).handle(msg)

        def _on_state(self, state, ident):
            log.append(("pending", ident[0]))
            super(Master, self)._on_state(state, ident)

    master = Master(c2s, s2c, n, batch_policy=batch_policy, max_wait=0.01)
    procs = S.start_simulators(S.SyntheticSimulatorWorker, n, c2s, s2c, seed=200)
    master.start()
    t0 = time.time()
    while len(master.queue) < 300 and time.time() - t0 < 60:
        time.sleep(0.02)
    master.stop()
    master.join(timeout=30)
    for p in procs:
        p.join(timeout=30)
    master.close()
    assert not master.is_alive() and master.is_done
    assert all(p.exitcode == 0 for p in procs)
    assert len(master.queue) >= 300
    assert max(master.round_sizes) > 1 and max(master.round_sizes) <= n   # real batching

    # replay: messages update memories in arrival order; a round's decisions are applied in
    # the order its states were queued (== the mirror's on_state order)
    mirror = O.SimulatorMasterMirror()
    pend = []
    for e in log:
        if e[0] == "msg":
            mirror.on_message(e[1], e[2], e[3])
        elif e[0] == "pending":
            pend.append(e[1])
        else:
            _, sums, acts, vals = e
            assert len(sums) == len(pend)
            for ident, ssum, a, v in zip(pend, sums, acts, vals):
                mirror.on_state(ident, ssum, a, v)
            pend = []
    got = master.queue[:len(mirror.queue)]
    assert len(mirror.queue) == len(master.queue)
    for (st, act, R, ts, init_r, over), (tr, R_ref, init_ref, over_ref) in zip(got, mirror.queue):
        assert int(st.sum()) == tr["state"] and act == tr["action"]
        assert R == R_ref and float(init_r) == float(init_ref) and over == over_ref
    # the decisions are one RandomState stream consumed in arrival order
    rs2 = np.random.RandomState(21)
    for e in log:
        if e[0] == "round":
            for ssum, a in zip(e[1], e[2]):
                p = [0.1, 0.2, 0.3, 0.4] if ssum % 2 else [0.25] * 4
                assert rs2.choice(4, p=p) == a
