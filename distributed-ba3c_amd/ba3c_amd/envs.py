"""Players of the simulator side: the RLEnvironment / ProxyPlayer
contract (RL/envbase.py:13-141) and the wrappers OpenAIGym/train.py:113-128 stacks around the
game (RL/history.py:12-55, RL/common.py:14-83).

They run inside each simulator process on the host, exactly where the reference runs them;
only their states cross into the learner (ba3c_amd.simulator).  gym/ALE are not installable
here, so `SyntheticAtariPlayer` stands in for GymEnv + the 84x84 resize (grayscale uint8
frames, integer rewards incl. values the returns clip, episodes of 20..80 steps).
"""
from collections import defaultdict, deque

import numpy as np

FRAME_HISTORY = 4          # train.py:95 (--frame_history default)
IMAGE_SIZE = (84, 84)      # train.py:92


class DiscreteActionSpace(object):
    """RL/envbase.py:108-124: `sample()` draws from the space's own RNG."""

    def __init__(self, num, seed=None):
        self.num = int(num)
        self.rng = np.random.RandomState(seed)

    def sample(self):
        return self.rng.randint(self.num)

    def num_actions(self):
        return self.num

    def __repr__(self):
        return "DiscreteActionSpace({})".format(self.num)


class RLEnvironment(object):
    """RL/envbase.py:13-72."""

    def __init__(self):
        self.reset_stat()

    def current_state(self):
        raise NotImplementedError()

    def action(self, act):
        """Perform `act`; returns (reward, isOver).  Starts a new episode when isOver."""
        raise NotImplementedError()

    def restart_episode(self):
        raise NotImplementedError()

    def finish_episode(self):
        pass

    def get_action_space(self):
        raise NotImplementedError()

    def reset_stat(self):
        self.stats = defaultdict(list)

    def play_one_episode(self, func, stat="score"):
        """envbase.py:54-72: run `func(state) -> action` until the episode ends."""
        if not isinstance(stat, list):
            stat = [stat]
        while True:
            s = self.current_state()
            r, over = self.action(func(s))
            if over:
                out = [self.stats[k] for k in stat]
                self.reset_stat()
                return out if len(out) > 1 else out[0]


class ProxyPlayer(RLEnvironment):
    """RL/envbase.py:126-155: forwards everything to `player`."""

    def __init__(self, player):
        self.player = player

    def reset_stat(self):
        self.player.reset_stat()

    def current_state(self):
        return self.player.current_state()

    def action(self, act):
        return self.player.action(act)

    @property
    def stats(self):
        return self.player.stats

    def restart_episode(self):
        self.player.restart_episode()

    def finish_episode(self):
        self.player.finish_episode()

    def get_action_space(self):
        return self.player.get_action_space()


class HistoryFramePlayer(ProxyPlayer):
    """RL/history.py:12-55: the state is the last `hist_len` frames concatenated on the
    channel axis, zero frames in front at the start of an episode."""

    def __init__(self, player, hist_len):
        super(HistoryFramePlayer, self).__init__(player)
        self.history = deque(maxlen=hist_len)
        self.history.append(self._frame())

    def _frame(self):
        s = self.player.current_state()
        return s.reshape(s.shape[0], s.shape[1], 1) if s.ndim != 3 else s

    def current_state(self):
        assert len(self.history) != 0
        pad = [np.zeros_like(self.history[0])] * (self.history.maxlen - len(self.history))
        return np.concatenate(pad + list(self.history), axis=2)

    def action(self, act):
        r, over = self.player.action(act)
        s = self._frame()
        self.history.append(s)
        if over:                              # s is the first frame of a new episode
            self.history.clear()
            self.history.append(s)
        return r, over

    def restart_episode(self):
        super(HistoryFramePlayer, self).restart_episode()
        self.history.clear()
        self.history.append(self._frame())


class PreventStuckPlayer(ProxyPlayer):
    """RL/common.py:14-40: after `nr_repeat` identical actions in a row, play `action`
    instead (e.g. FIRE to start Breakout).  The repeat window is cleared on episode end."""

    def __init__(self, player, nr_repeat, action):
        super(PreventStuckPlayer, self).__init__(player)
        self.act_que = deque(maxlen=nr_repeat)
        self.trigger_action = action

    def action(self, act):
        self.act_que.append(act)
        if self.act_que.count(self.act_que[0]) == self.act_que.maxlen:
            act = self.trigger_action
        r, over = self.player.action(act)
        if over:
            self.act_que.clear()
        return r, over

    def restart_episode(self):
        super(PreventStuckPlayer, self).restart_episode()
        self.act_que.clear()


class LimitLengthPlayer(ProxyPlayer):
    """RL/common.py:42-64: end (and restart) the episode after `limit` actions."""

    def __init__(self, player, limit):
        super(LimitLengthPlayer, self).__init__(player)
        self.limit = limit
        self.cnt = 0

    def action(self, act):
        r, over = self.player.action(act)
        self.cnt += 1
        if self.cnt >= self.limit:
            over = True
            self.finish_episode()
            self.restart_episode()
        if over:
            self.cnt = 0
        return r, over

    def restart_episode(self):
        self.player.restart_episode()
        self.cnt = 0


class AutoRestartPlayer(ProxyPlayer):
    """RL/common.py:66-74: finish + restart the underlying player on episode end."""

    def action(self, act):
        r, over = self.player.action(act)
        if over:
            self.player.finish_episode()
            self.player.restart_episode()
        return r, over


class MapPlayerState(ProxyPlayer):
    """RL/common.py:76-83: `current_state` passed through `func` (train.py:116-119 resizes)."""

    def __init__(self, player, func):
        super(MapPlayerState, self).__init__(player)
        self.func = func

    def current_state(self):
        return self.func(self.player.current_state())


class SyntheticAtariPlayer(RLEnvironment):
    """Stand-in for GymEnv (gym/ALE absent): one game whose frame at step t is a moving byte
    pattern, reward 1 when the action matches a per-step target (3 every 7th step, which the
    returns clip), episodes of 20..80 steps; auto-restarts like GymEnv and records the
    episode 'score' stat the evaluation reads."""

    def __init__(self, idx=0, num_actions=4, seed=0):
        super(SyntheticAtariPlayer, self).__init__()
        self.idx = int(idx)
        self.A = int(num_actions)
        self.rng = np.random.RandomState(seed)
        self.space = DiscreteActionSpace(self.A, seed=seed + 1)
        yy, xx = np.mgrid[0:IMAGE_SIZE[0], 0:IMAGE_SIZE[1]]
        self._base = 3 * xx + 5 * yy
        self.restart_episode()

    def restart_episode(self):
        self.t = 0
        self.length = int(self.rng.randint(20, 81))
        self.score = 0.0

    def finish_episode(self):
        self.stats["score"].append(self.score)

    def current_state(self):
        return ((self._base + 7 * self.t + 11 * self.idx) & 255).astype(np.uint8)

    def action(self, act):
        hit = float(int(act) == (self.t + self.idx) % self.A)
        r = 3.0 * hit if self.t % 7 == 6 else hit
        self.score += r
        self.t += 1
        over = self.t >= self.length
        if over:
            self.finish_episode()
            self.restart_episode()
        return r, over

    def get_action_space(self):
        return self.space


def get_player(idx=0, num_actions=4, seed=0, train=False, frame_history=FRAME_HISTORY,
               limit=40000):
    """OpenAIGym/train.py:113-128 with the synthetic game: history of `frame_history` frames,
    PreventStuckPlayer(30, 1) for evaluation players, LimitLengthPlayer(40000)."""
    pl = SyntheticAtariPlayer(idx, num_actions, seed)
    pl = HistoryFramePlayer(pl, frame_history)
    if not train:
        pl = PreventStuckPlayer(pl, 30, 1)
    return LimitLengthPlayer(pl, limit)
