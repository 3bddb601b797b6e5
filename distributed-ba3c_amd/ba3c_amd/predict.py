"""Predictor path: OnlinePredictor (predict/base.py:72-92), DummyOnlinePredictor (:94-105) and
the MultiThreadAsyncPredictor (predict/concurrency.py:82-219), re-designed as ONE large-batch
GPU forward.

The reference answers each simulator state with a <=16-state micro-batch on 3 CPU threads;
here queued states are concatenated and forwarded in a single `ba3c_forward` launch chain on
the predictor's HIP stream (so it overlaps the learner's stream), and actions are sampled on
that same stream with numpy-exact semantics from host-drawn MT19937 uniforms (train.py:382).
The evaluation players' greedy choice (OpenAIGym/common.py:24-33) is `greedy_actions`.
"""
import contextlib
import queue
import threading

import numpy as np
import torch


class OnlinePredictor(object):
    """f([states]) -> [logitsT, pred_value, global_step, True] (predict/base.py:80-92);
    on failure returns dummy outputs and the False flag like the reference (:86-91).

    With `stream` set, the forward (and everything MultiThreadAsyncPredictor does with its
    outputs) runs on that HIP stream; the returned device tensors are valid on it."""

    def __init__(self, model, input_names=("state",), output_names=("logitsT", "pred_value"),
                 stream=None):
        self.model = model
        self.engine = model.engine
        self.input_names = list(input_names)
        self.output_names = list(output_names)
        self.stream = stream
        self.global_step = 0

    def on_stream(self):
        """Context that makes the predictor's stream current (a no-op without one)."""
        if self.stream is None:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.stream)

    def _forward(self, states):
        eng = self.engine
        if isinstance(states, np.ndarray):
            states = torch.from_numpy(np.ascontiguousarray(states, dtype=np.uint8))
        states = states.to(eng.device, non_blocking=True).contiguous()
        probs, probsT, value = eng.forward(states, explore_factor=self.model.explore_factor)
        outs = {"logits": probs, "logitsT": probsT, "pred_value": value}
        return [outs[n] for n in self.output_names]

    def __call__(self, dp):
        states = dp[0]
        try:
            with self.on_stream():
                outs = self._forward(states)
            return outs + [self.global_step, True]
        except Exception:
            n = len(states)
            return [np.zeros((n, self.engine.num_actions), np.float32), np.zeros(n, np.float32),
                    0, False]


class DummyOnlinePredictor(object):
    """--dummy_predictor (predict/base.py:94-105, selected at train/trainer.py:50-51): uniform
    policy over the actions and U(0,1) values, no network evaluation."""

    def __init__(self, num_actions, rs=None):
        self.num_actions = num_actions
        self.rs = rs if rs is not None else np.random
        self.global_step = 0
        self.engine = None

    def on_stream(self):
        return contextlib.nullcontext()

    def __call__(self, dp):
        z = len(dp[0])
        probs = np.full((z, self.num_actions), 1.0 / self.num_actions, np.float32)
        return [probs, self.rs.uniform(size=(z, 1)), self.global_step, True]


class MultiThreadAsyncPredictor(object):
    """Queue of single-state tasks served in large batches (concurrency.py:172-219).

    put_task([state], callback) enqueues; a worker thread drains up to `batch_size` tasks,
    runs one GPU forward + GPU sampling, and calls each callback with
    [probs_i, value_i, global_step, True, action_i]; when the forward fails every callback of
    the batch receives [False] (concurrency.py:144-146, handled at train.py:385-387).
    `rs` is the numpy RandomState whose uniform stream np.random.choice would consume (one
    double per state, in order)."""

    def __init__(self, predictor, batch_size=8192, rs=None):
        self.predictor = predictor
        self.batch_size = batch_size
        self.rs = rs if rs is not None else np.random.RandomState(0)
        self.tasks = queue.Queue()
        self._stop = threading.Event()
        self._thread = None

    def put_task(self, dp, callback=None):
        self.tasks.put((dp, callback))

    def run(self):
        self._thread = threading.Thread(target=self._loop, daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join()

    def _fetch_batch(self):
        first = self.tasks.get(timeout=0.1)
        batch = [first]
        while len(batch) < self.batch_size:
            try:
                batch.append(self.tasks.get_nowait())
            except queue.Empty:
                break
        return batch

    def predict_batch(self, states):
        """One forward of [b,84,84,C] states + sampling on the predictor's stream; returns
        host (probs, values, actions), or None when the forward reported failure."""
        out = self.predictor([states])
        if not out[-1]:
            return None
        probs, value = out[0], out[1]
        eng = self.predictor.engine
        with self.predictor.on_stream():        # sampling reads probs on the stream that wrote them
            # one MT19937 double per state, drawn in one call: the same stream as len(states)
            # scalar random_sample() calls (train.py:382 draws one per np.random.choice)
            u = torch.from_numpy(self.rs.random_sample(len(states))).to(eng.device)
            actions, flag = eng.sample(probs, u)
            f = int(flag.item())
            if f & 1:
                raise AssertionError("non-finite action distribution (train.py:381)")
            if f & (2 | 4):
                raise ValueError("probabilities do not sum to 1 / are negative")
            return probs.cpu().numpy(), value.cpu().numpy(), actions.cpu().numpy()

    def _loop(self):
        while not self._stop.is_set():
            try:
                batch = self._fetch_batch()
            except queue.Empty:
                continue
            states = np.stack([np.asarray(dp[0]) for dp, _ in batch])
            res = self.predict_batch(states)
            for i, (_, cb) in enumerate(batch):
                if cb is None:
                    continue
                if res is None:
                    cb([False])
                else:
                    probs, values, actions = res
                    cb([probs[i], values[i], self.predictor.global_step, True, int(actions[i])])


def greedy_actions(engine, probs, u, random_actions, eps=0.001):
    """Evaluation players' choice (OpenAIGym/common.py:24-33): argmax of the policy (first
    maximum, numpy's argmax), replaced by `random_actions[i]` (the action space's sample)
    where u[i] < eps (`random.random() < 0.001`).  probs: device [B,A] fp32; u: device
    float64 [B]; random_actions: device int64 [B].  Runs as one HIP kernel."""
    return engine.greedy(probs, u, random_actions, eps)
