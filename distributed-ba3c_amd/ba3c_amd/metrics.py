"""Training metrics with the reference's scalar names and CSV channels.

DebugLogCallback (OpenAIGym/common.py:172-288) averages the step dictionaries (`TfDictOp`
results, train/multigpu.py:193-205) over --send_debug_every steps and sends the reference's
message tuples ('loss', cost, policy_loss, xentropy_loss, value_loss, advantage, pred_reward,
max_logit), ('other', active_relus, dp_per_s) and ('delays', (mean, max, min)); the
CsvChannels sink replaces the Neptune metrics server's _dump_to_channels
(neptune_mp_server.py:169-233) writing one `<channel>.csv` ("x,y" rows, x = hours since start)
per channel as utils/neptune_utils.py:38-57 does.
"""
import os
import time

import numpy as np


class StatCounter(object):
    """utils/stat.py:8-39."""

    def __init__(self):
        self.reset()

    def feed(self, v):
        self._values.append(v)

    def reset(self):
        self._values = []

    @property
    def count(self):
        return len(self._values)

    @property
    def average(self):
        assert len(self._values)
        return np.mean(self._values)

    @property
    def sum(self):
        assert len(self._values)
        return np.sum(self._values)

    @property
    def max(self):
        assert len(self._values)
        return max(self._values)


class CsvChannels(object):
    """The chief's metrics sink: Server._dump_to_channels onto `<name>.csv` channel files."""

    LOSS = ["cost", "policy_loss", "xentropy_loss", "value_loss", "advantage", "pred_reward",
            "max_logit"]

    def __init__(self, experiment_dir):
        self.dir = experiment_dir
        os.makedirs(experiment_dir, exist_ok=True)
        self.start = time.time()
        self._fd = {}

    def _send(self, name, x, y):
        fd = self._fd.get(name)
        if fd is None:
            fd = self._fd[name] = open(os.path.join(self.dir, name + ".csv"), "w")
            fd.write("x,y\n")
        fd.write("{},{}\n".format(x, y))
        fd.flush()

    def send(self, message):
        _, content = message
        x = (time.time() - self.start) / 3600.0
        kind = content[0]
        if kind == "loss":
            for name, v in zip(self.LOSS, content[1:]):
                self._send(name, x, v)
        elif kind == "other":
            self._send("active_relus", x, content[1])
            self._send("dp_per_s", x, content[2])
        elif kind == "delays":
            mean, mx, mn = content[1]
            self._send("mean_delay", x, mean)
            self._send("max_delay", x, mx)
            self._send("min_delay", x, mn)
        elif kind == "score":
            self._send("score_mean", x, content[1])
            self._send("score_max", x, content[2])
        elif kind == "online":
            self._send("online_score", x, content[1])

    def close(self):
        for fd in self._fd.values():
            fd.close()
        self._fd = {}


class DebugLogCallback(object):
    """OpenAIGym/common.py:172-288 (the default, non-debug-chart messages)."""

    def __init__(self, client, worker_id=0, nr_send=100):
        self.client, self.worker_id, self.send_every = client, worker_id, int(nr_send)
        self.dp_per_s = StatCounter()
        self.lists = None
        self.delays = []
        self.counter = 0
        self.step_counter = 0

    def trigger_step(self, session_result, dp_per_s, delay=None):
        if self.lists is None:
            self.lists = {name: StatCounter() for name in session_result}
        for name in session_result:
            self.lists.setdefault(name, StatCounter()).feed(session_result[name])
        self.dp_per_s.feed(dp_per_s)
        if delay is not None:
            self.delays.append(delay)
        self.counter += 1
        self.step_counter += 1
        if self.counter < self.send_every:
            return False
        L = self.lists
        self.client.send((self.worker_id, ("loss",) + tuple(
            float(L[k].average) for k in CsvChannels.LOSS)))
        self.client.send((self.worker_id, ("other", float(L["active_relus"].average),
                                           float(self.dp_per_s.average))))
        if self.delays:
            d = np.asarray(self.delays, np.float64)
            self.client.send((self.worker_id, ("delays", (float(np.mean(d)), float(np.max(d)),
                                                          float(np.min(d))))))
        self.counter = 0
        for s in self.lists.values():
            s.reset()
        self.dp_per_s.reset()
        self.delays = []
        return True
