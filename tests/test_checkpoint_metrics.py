"""Checkpoint format (ModelSaver / SaverRestore / ParamRestore with the reference's variable
names) and the metrics channels (DebugLogCallback -> CSV channels,
rank 4)."""
import os

import numpy as np
import pytest
import torch

from oracle import ba3c_oracle as O


def test_debug_log_callback_writes_reference_channels(tmp_path):
    from ba3c_amd.metrics import CsvChannels, DebugLogCallback
    sink = CsvChannels(str(tmp_path))
    cb = DebugLogCallback(sink, worker_id=0, nr_send=3)
    keys = ["cost", "policy_loss", "xentropy_loss", "value_loss", "advantage", "pred_reward",
            "max_logit", "active_relus"]
    sent = []
    for i in range(6):
        sent.append(cb.trigger_step({k: float(i + j) for j, k in enumerate(keys)},
                                    dp_per_s=100.0 * i, delay=float(i)))
    sink.close()
    assert sent == [False, False, True, False, False, True]
    rows = open(os.path.join(str(tmp_path), "cost.csv")).read().strip().split("\n")
    assert rows[0] == "x,y" and [float(r.split(",")[1]) for r in rows[1:]] == [1.0, 4.0]
    dps = open(os.path.join(str(tmp_path), "dp_per_s.csv")).read().strip().split("\n")
    assert [float(r.split(",")[1]) for r in dps[1:]] == [100.0, 400.0]
    for ch in ("policy_loss", "xentropy_loss", "value_loss", "advantage", "pred_reward",
               "max_logit", "active_relus", "mean_delay", "max_delay", "min_delay"):
        assert os.path.exists(os.path.join(str(tmp_path), ch + ".csv")), ch


def _trainer(seed=0):
    from ba3c_amd.model import Model
    from ba3c_amd.optimizer import AdamOptimizer
    from ba3c_amd.trainer import Ba3cTrainer, TrainConfig
    m = Model(num_actions=4, fc_neurons=128, fc_splits=4, batch_size=16, max_batch=16)
    m.engine.load_params(O.init_params(128, 4, 4, seed=seed, dtype=np.float32))
    return Ba3cTrainer(TrainConfig(model=m, optimizer=AdamOptimizer(1e-3, 0.8, 0.75, 1e-8)))


def _batch(i):
    rs = np.random.RandomState(50 + i)
    return (torch.from_numpy(rs.randint(0, 256, size=(16, 84, 84, 4)).astype(np.uint8)).cuda(),
            torch.from_numpy(rs.randint(0, 4, size=16).astype(np.int64)).cuda(),
            torch.from_numpy(rs.normal(size=16).astype(np.float32)).cuda())


@pytest.mark.gpu
def test_resume_from_checkpoint_is_bit_exact(tmp_path):
    from ba3c_amd.checkpoint import ModelSaver, PeriodicPerStepCallback, SaverRestore
    a = _trainer()
    saver = PeriodicPerStepCallback(ModelSaver(str(tmp_path)), 3)
    path = None
    for i in range(3):
        a.train_step(*_batch(i))
        path = saver.trigger_step(a) or path
    assert path and os.path.basename(os.path.dirname(path)) == "iter_0"
    with np.load(path, allow_pickle=False) as f:
        names = set(f.files)
        assert {n for n, _ in O.param_specs(128, 4, 4)} <= names
        assert {"conv0/W/Adam", "conv0/W/Adam_1", "beta1_power", "beta2_power", "global_step"} <= names
        assert f["conv0/W"].shape == (5, 5, 16, 32) and int(f["global_step"]) == 3
    b = _trainer(seed=9)                       # different init: everything must come from the file
    SaverRestore(path).init(b)
    assert b.global_step == 3
    for i in range(3, 5):
        a.train_step(*_batch(i))
        b.train_step(*_batch(i))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.engine.params.cpu().numpy(), b.engine.params.cpu().numpy())
    for sa, sb in zip(a.optimizer.slots, b.optimizer.slots):
        np.testing.assert_array_equal(sa.cpu().numpy(), sb.cpu().numpy())


@pytest.mark.gpu
def test_param_restore_from_dict_by_reference_names():
    from ba3c_amd.checkpoint import ParamRestore
    t = _trainer()
    p = O.init_params(128, 4, 4, seed=4, dtype=np.float32)
    used = ParamRestore({k + ":0": v for k, v in p.items()}).init(t)
    assert used == set(p)
    got = t.engine.state_dict()
    for k in p:
        np.testing.assert_array_equal(got[k], p[k])
