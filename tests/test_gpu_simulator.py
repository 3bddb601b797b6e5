"""Simulator side on the GPU: BatchedSimulatorMaster answers each round
of simulator messages with ONE predictor forward of the whole round + numpy-exact sampling
(train.py:355-437 / predict/concurrency.py:172-219 re-designed).  Its datapoints must equal
the oracle's restatement of the per-message master replayed on the same message log, its
policy outputs must match the oracle forward, and its actions must be np.random.choice draws
of one RandomState over the GPU probabilities in arrival order."""
import os
import tempfile
import time

import numpy as np
import pytest

from oracle import ba3c_oracle as O

pytestmark = pytest.mark.gpu


def test_batched_master_over_ipc_with_gpu_predictor():
    from ba3c_amd import simulator as S
    from ba3c_amd.model import Model
    from ba3c_amd.predict import OnlinePredictor
    from ba3c_amd.simulator_gpu import BatchedSimulatorMaster

    n = 6
    m = Model(num_actions=4, channels=1, fc_neurons=128, fc_splits=4, batch_size=n, max_batch=n)
    p32 = O.init_params(128, 4, 4, seed=8, dtype=np.float32)
    m.engine.load_params(p32)
    p64 = {k: v.astype(np.float64) for k, v in p32.items()}
    log = []

    class Master(BatchedSimulatorMaster):
        def handle(self, msg):
            ident, state, reward, is_over, ts, alive = msg
            if alive and not self._stop_req.is_set():
                log.append(("msg", ident, float(reward), bool(is_over)))
            return super(Master, self).handle(msg)

        def _on_state(self, state, ident):
            log.append(("pending", ident[0], np.array(state)))
            super(Master, self)._on_state(state, ident)

        def _flush(self):
            k = len(self._pending)
            super(Master, self)._flush()
            if k:
                idents = [e[1] for e in log if e[0] == "pending"][-k:]
                mem = [self.clients[i].memory[-1] for i in idents]
                log.append(("round", [(t.action, t.value) for t in mem]))

    d = tempfile.mkdtemp(prefix="ba3c_ipcg_")
    c2s, s2c = "ipc://" + os.path.join(d, "c2s"), "ipc://" + os.path.join(d, "s2c")
    master = Master(c2s, s2c, n, predictor=OnlinePredictor(m), rs=np.random.RandomState(5),
                    max_wait=0.01)
    # threads, not processes: this process already holds the GPU
    S.start_simulators(S.SyntheticSimulatorWorker, n, c2s, s2c, threads=True, seed=300)
    master.start()
    t0 = time.time()
    while len(master.queue) < 200 and time.time() - t0 < 90:
        time.sleep(0.02)
    master.stop()
    master.join(timeout=30)
    master.close()
    assert master.is_done and len(master.queue) >= 200
    assert max(master.round_sizes) > 1

    mirror = O.SimulatorMasterMirror()
    pend, states, acts, probs_ref = [], [], [], []
    for e in log:
        if e[0] == "msg":
            mirror.on_message(e[1], e[2], e[3])
        elif e[0] == "pending":
            pend.append((e[1], e[2]))
        else:
            assert len(e[1]) == len(pend)
            for (ident, st), (a, v) in zip(pend, e[1]):
                mirror.on_state(ident, int(st.sum()), a, v)
                states.append(st)
                acts.append(a)
            pend = []
    got = master.queue[:len(mirror.queue)]
    assert len(mirror.queue) == len(master.queue)
    for (st, act, R, ts, init_r, over), (tr, R_ref, init_ref, over_ref) in zip(got, mirror.queue):
        assert int(st.sum()) == tr["state"] and act == tr["action"]
        assert R == R_ref and float(init_r) == float(init_ref) and over == over_ref

    # policy outputs vs the oracle forward, and actions = numpy choice over the GPU
    # probabilities with the master's RandomState stream (arrival order)
    import torch
    states = np.stack(states)
    probs_gpu = np.concatenate([m.engine.forward(torch.from_numpy(states[i:i + n]).cuda())[1].cpu().numpy()
                                for i in range(0, len(states), n)])
    np.testing.assert_array_equal(np.array(acts), O.np_random_choice(probs_gpu, np.random.RandomState(5)))
    k = 24                                     # oracle (fp64 numpy) check on the first rounds
    t = O.get_nn_prediction(p64, states[:k], {"fc_neurons": 128, "fc_splits": 4})
    vals = np.array([v for e in log if e[0] == "round" for (_, v) in e[1]])[:k]
    vscale = ((np.abs(t["h"]) @ np.abs(p64["fc-v/W"]))[:, 0] + abs(p64["fc-v/b"][0])).max()
    assert np.abs(vals - t["pred_value"]).max() / vscale < 1e-5
    assert np.abs(probs_gpu[:k] - t["logitsT"]).max() < 1e-5
