"""End-to-end BA3C actor-learner loop on one GPU (BASELINE configs[0] "plumbing": the
reference's 1 worker + 1 PS Breakout run, with a synthetic environment in place of gym/ALE,
which are not installable here).

One iteration is the reference's per-simulator message cycle (RL/simulator.py:95-109,
:160-185 and MySimulatorMaster, OpenAIGym/train.py:364-437) for every simulator at once:

  state (FrameHistory, RL/history.py) -> predictor forward ('logitsT', 'pred_value') ->
  action = np.random.choice semantics on the GPU from host MT19937 draws (train.py:382) ->
  RolloutBuffer.on_state -> env step -> FrameHistory.push -> RolloutBuffer.on_reward
  (n-step returns, train.py:408-437) -> BatchQueue (BatchData) -> Ba3cTrainer.train_step

The synthetic environment is NOT part of the reference's hot path; it only produces frames,
rewards and episode ends with the shapes and value ranges of the Atari pipeline (84x84
grayscale frames, integer rewards incl. values outside [-1, 1] that the returns clip).
"""
import numpy as np
import torch

from .rollout import BatchQueue, FrameHistory, RolloutBuffer


class SyntheticAtari(object):
    """E simulators on the device: frame_e(t) is a moving byte pattern, the reward is 1 when
    the action matches a per-step target (3 every 7th step: clipped by the returns), episodes
    last 20..80 steps."""

    def __init__(self, n_envs, num_actions=4, seed=0, device="cuda"):
        self.E, self.A = int(n_envs), int(num_actions)
        self.device = torch.device(device)
        self.g = torch.Generator(device=self.device).manual_seed(seed)
        self.t = torch.zeros(self.E, dtype=torch.int64, device=self.device)
        self.L = self._lengths()
        yy = torch.arange(84, device=self.device).view(1, 84, 1)
        xx = torch.arange(84, device=self.device).view(1, 1, 84)
        self._base = (3 * xx + 5 * yy)                       # [1,84,84]
        self._eid = torch.arange(self.E, device=self.device).view(-1, 1, 1)

    def _lengths(self):
        return torch.randint(20, 81, (self.E,), generator=self.g, device=self.device)

    def frames(self):
        f = (self._base + 7 * self.t.view(-1, 1, 1) + 11 * self._eid) & 255
        return f.to(torch.uint8).unsqueeze(-1).contiguous()     # [E,84,84,1]

    def step(self, actions):
        target = (self.t + torch.arange(self.E, device=self.device)) % self.A
        hit = (actions.to(torch.int64) == target).to(torch.float64)
        reward = torch.where(self.t % 7 == 6, 3.0 * hit, hit)
        self.t += 1
        over = self.t >= self.L
        if bool(over.any()):
            newL = self._lengths()
            self.L = torch.where(over, newL, self.L)
            self.t = torch.where(over, torch.zeros_like(self.t), self.t)
        return self.frames(), reward, over


class ActorLearner(object):
    """The loop above around an existing Ba3cTrainer (whose model engine also serves as the
    predictor: the reference's towerp0 reads the same variables, train.py:355-362)."""

    def __init__(self, trainer, n_envs, batch_size, seed=0, rs=None, on_train_step=None,
                 dummy_predictor=False):
        """on_train_step(trainer): called after every learner step (callbacks / metrics);
        dummy_predictor: --dummy_predictor 1 (predict/base.py:94-105) — uniform policy and
        U(0,1) values instead of the network forward."""
        eng = trainer.engine
        assert eng.channels == 4, "synthetic loop is grayscale x FRAME_HISTORY=4"
        self.trainer = trainer
        self.engine = eng
        self.env = SyntheticAtari(n_envs, eng.num_actions, seed=seed, device=eng.device)
        self.hist = FrameHistory(n_envs, hist_len=4, channels=1, device=eng.device)
        self.buf = RolloutBuffer(n_envs, channels=4, device=eng.device)
        self.queue = BatchQueue(batch_size)
        self.rs = rs if rs is not None else np.random.RandomState(seed)
        self.hist.push(self.env.frames(), torch.ones(n_envs, dtype=torch.bool, device=eng.device))
        self.steps = 0
        self.train_steps = 0
        self.last_scalars = None
        self.on_train_step = on_train_step
        self.dummy_predictor = dummy_predictor

    def _predict(self, state):
        eng = self.engine
        if self.dummy_predictor:
            E, A = self.env.E, eng.num_actions
            probs = torch.full((E, A), 1.0 / A, dtype=torch.float32, device=eng.device)
            value = torch.from_numpy(self.rs.uniform(size=E).astype(np.float32)).to(eng.device)
            return probs, value
        _, probsT, value = eng.forward(state, explore_factor=self.trainer.model.explore_factor)
        return probsT, value

    def iterate(self):
        eng = self.engine
        state = self.hist.state
        probsT, value = self._predict(state)
        u = torch.from_numpy(self.rs.random_sample(self.env.E)).to(eng.device)
        actions, flag = eng.sample(probsT, u)
        self.buf.on_state(state, actions, value)
        frames, reward, over = self.env.step(actions)
        self.hist.push(frames, over)
        self.queue.put(self.buf.on_reward(reward, over))
        while True:
            b = self.queue.get()
            if b is None:
                break
            self.trainer.train_step(b[0].contiguous(), b[1].contiguous(), b[2].contiguous())
            self.train_steps += 1
            self.last_scalars = self.trainer.model.scalars
            if self.on_train_step is not None:
                self.on_train_step(self.trainer)
        self.steps += 1
        if int(flag.item()) & 1:
            raise AssertionError("non-finite action distribution (train.py:381)")

    def run(self, n):
        for _ in range(n):
            self.iterate()
        return self
