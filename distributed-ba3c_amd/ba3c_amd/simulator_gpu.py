"""BatchedSimulatorMaster — the simulator master of RL/simulator.py:114-200 with
MySimulatorMaster's callbacks (OpenAIGym/train.py:355-437), re-designed around ONE batched
predictor call per round.

The reference answers each simulator's state on its own: `_on_state` queues one task on the
MultiThreadAsyncPredictor (predict/concurrency.py:172-219), whose threads forward <= 16 states
on the CPU and call back `np.random.choice(len(distrib), p=distrib)` (train.py:374-390) per
state.  Here one round collects the pending message of every simulator that has one (each
simulator waits for its reply before it sends again, so a round holds at most one message per
simulator and no two of its messages touch the same client memory), runs the per-message
memory logic of the reference (`SimulatorMaster.handle`: reward of the previous transition,
episode end / n-step parse) in arrival order, and then answers every state of the round with
ONE call of `batch_policy(states) -> (probs, values, actions)` — on the GPU that is
`MultiThreadAsyncPredictor.predict_batch`: one `ba3c_forward` of the whole round plus
numpy-exact sampling on the predictor's stream, the uniforms drawn from `rs` in arrival order.
Replies, memory entries (TransitionExperience(state, action, None, value=..., ts=...)) and
datapoints are exactly those of the per-message master given the same decisions.
"""
import numpy as np

from .simulator import SimulatorMaster, TransitionExperience, loads


class BatchedSimulatorMaster(SimulatorMaster):
    """`batch_policy(states [b,84,84,C] uint8) -> (probs [b,A], values [b], actions [b])`,
    or `predictor` (an OnlinePredictor; its MultiThreadAsyncPredictor.predict_batch is used,
    drawing from `rs`).  `max_wait` seconds: how long a round waits for more messages after
    its first one (0: only what has already arrived)."""

    def __init__(self, pipe_c2s, pipe_s2c, simulator_procs, batch_policy=None, predictor=None,
                 rs=None, max_wait=0.002, **kw):
        super(BatchedSimulatorMaster, self).__init__(pipe_c2s, pipe_s2c, simulator_procs, **kw)
        if (batch_policy is None) == (predictor is None):
            raise ValueError("give exactly one of batch_policy / predictor")
        if predictor is not None:
            from .predict import MultiThreadAsyncPredictor
            async_pred = MultiThreadAsyncPredictor(predictor, rs=rs)

            def batch_policy(states):
                res = async_pred.predict_batch(states)
                if res is None:
                    raise RuntimeError("predictor forward failed")
                return res
        self.batch_policy = batch_policy
        self.max_wait = float(max_wait)
        self.global_step = 0
        self.rounds = 0
        self.round_sizes = []
        self._pending = []

    def _on_state(self, state, ident):
        """Deferred to the round's single batched decision (train.py:374-390)."""
        self._pending.append((state, ident))

    def _flush(self):
        if not self._pending:
            return
        states = np.stack([np.asarray(s, dtype=np.uint8) for s, _ in self._pending])
        probs, values, actions = self.batch_policy(states)
        probs = np.asarray(probs)
        assert np.all(np.isfinite(probs)), probs          # train.py:381
        for i, (state, (ident, ts)) in enumerate(self._pending):
            action = int(actions[i])
            self.clients[ident].memory.append(
                TransitionExperience(state, action, None, value=float(np.asarray(values[i]).reshape(-1)[0]),
                                     ts=ts))
            self.send(ident, action, self.global_step)
        self.rounds += 1
        self.round_sizes.append(len(self._pending))
        self._pending = []

    def run(self):
        while True:
            buf = self.c2s_socket.recv(timeout=1.0)
            if buf is None:
                continue
            bufs = [buf]
            while len(bufs) < self.simulator_procs:
                nxt = self.c2s_socket.recv(timeout=self.max_wait)
                if nxt is None:
                    break
                bufs.append(nxt)
            alive = True
            for b in bufs:
                self.messages += 1
                if not self.handle(loads(b)):
                    alive = False
                    break
            self._flush()
            if not alive:
                break
