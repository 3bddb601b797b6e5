"""Checkpoint save / restore with the reference's variable names.

ModelSaver (tensorpack callbacks/common.py:17-99, driven every --save_every steps by
PeriodicPerStepCallback, OpenAIGym/common.py:159-170, train.py:629-630) writes
`models_dir/iter_{i}/model-{hours}-{global_step}.npz`; SaverRestore / ParamRestore
(tfutils/sessinit.py:50-165) restore by name, warning — like the reference — about graph
variables missing from the file and file entries not in the graph.

Keys are the checkpoint names of train.py:180-264 (`conv0/W` ... `fc-v/b`) in TF layout
(HWIO convs, [in, out] FC), plus `global_step`.  Unlike the reference (weights only, Adam
restarts from zero on --load), the optimizer slots are saved under TF's slot names
(`<var>/Adam`, `<var>/Adam_1`, `beta1_power`, `beta2_power`; `<var>/RMSProp`,
`<var>/RMSProp_1`; ...) so a resumed run continues bit-exactly.  The format is a plain
`.npz` (no pickled objects; loaded with allow_pickle=False).
"""
import logging
import os
import time

import numpy as np

log = logging.getLogger("ba3c_amd.checkpoint")

# TF-1.2 slot names per optimizer (slot index -> suffix)
SLOT_NAMES = {"adam": ["Adam", "Adam_1"], "rms": ["RMSProp", "RMSProp_1"],
              "momentum": ["Momentum"], "adagrad": ["Adagrad"],
              "adadelta": ["Adadelta", "Adadelta_1"], "gd": []}


def _inner(opt):
    return getattr(opt, "_opt", opt)


def collect(trainer, with_slots=True):
    """{name: ndarray} of the trainer's model (+ optimizer state)."""
    eng = trainer.engine
    out = dict(eng.state_dict())
    out["global_step"] = np.int64(trainer.global_step)
    opt = _inner(trainer.optimizer)
    if with_slots and getattr(opt, "slots", None) is not None:
        for i, suffix in enumerate(SLOT_NAMES[opt.opt_id]):
            for k, v in eng.state_dict(opt.slots[i]).items():
                out["%s/%s" % (k, suffix)] = v
        if opt.opt_id == "adam":
            b1, b2 = opt.powers()
            out["beta1_power"], out["beta2_power"] = np.float32(b1), np.float32(b2)
    return out


def save(path, trainer, with_slots=True):
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    np.savez(path, **collect(trainer, with_slots))
    return path if path.endswith(".npz") else path + ".npz"


def restore(trainer, params, prefix=None):
    """Assign every graph variable found in `params` ({name: array}); returns the names used.
    Missing / unused names are logged like SaverRestore (sessinit.py:106-132)."""
    eng = trainer.engine
    key = (lambda n: "%s/%s" % (prefix, n)) if prefix else (lambda n: n)
    have = {}
    for n in eng.tensor_names:
        if key(n) in params:
            have[n] = np.asarray(params[key(n)], dtype=np.float32)
        else:
            log.warning("Variable %s in the graph not found in checkpoint!", n)
    cur = eng.state_dict()
    cur.update(have)
    eng.load_params(cur)
    used = {key(n) for n in have}
    if "global_step" in params:
        trainer.global_step = int(params["global_step"])
        used.add("global_step")
    opt = _inner(trainer.optimizer)
    suffixes = SLOT_NAMES.get(getattr(opt, "opt_id", "gd"), [])
    slot_keys = [k for k in params if any(k.endswith("/" + s) for s in suffixes)]
    if slot_keys:
        if opt.slots is None:
            opt.slots = opt._init_slots(eng)
        for i, suffix in enumerate(suffixes):
            vals = eng.state_dict(opt.slots[i])
            for n in eng.tensor_names:
                k = "%s/%s" % (key(n), suffix)
                if k in params:
                    vals[n] = np.asarray(params[k], dtype=np.float32)
                    used.add(k)
            flat = opt.slots[i]
            for n, off, numel, shape in eng.layout:
                import torch
                flat[off:off + numel].copy_(torch.from_numpy(np.ascontiguousarray(vals[n]).reshape(-1)))
        if getattr(opt, "opt_id", None) == "adam" and "beta1_power" in params:
            opt.beta1_power = np.float32(params["beta1_power"])
            opt.beta2_power = np.float32(params["beta2_power"])
            if opt.dev_powers is not None:
                opt.dev_powers.copy_(opt.dev_powers.new_tensor([opt.beta1_power, opt.beta2_power]))
            used.update(("beta1_power", "beta2_power"))
    for k in sorted(set(params) - used):
        log.warning("Variable %s in checkpoint not found in the graph!", k)
    return used


class SaverRestore(object):
    """tfutils/sessinit.py:50-132: restore a file written by ModelSaver."""

    def __init__(self, model_path, prefix=None):
        assert os.path.isfile(model_path), model_path
        self.path, self.prefix = model_path, prefix

    def init(self, trainer):
        with np.load(self.path, allow_pickle=False) as f:
            return restore(trainer, {k: f[k] for k in f.files}, self.prefix)


class ParamRestore(object):
    """tfutils/sessinit.py:134-165: restore from a {name: value} dict."""

    def __init__(self, param_dict):
        self.prms = {k[:-2] if k.endswith(":0") else k: v for k, v in param_dict.items()}

    def init(self, trainer):
        return restore(trainer, self.prms)


class ModelSaver(object):
    """callbacks/common.py:17-99 as a per-step callback: each trigger writes
    models_dir/iter_{i}/model-{hours since start}-{global_step}.npz (skipping an iter_ dir
    that is not empty, as the reference does)."""

    def __init__(self, models_dir, with_slots=True):
        self.models_dir = models_dir
        self.with_slots = with_slots
        self.i = 0
        self.start_time = time.time()
        self.path = None

    def trigger_step(self, trainer):
        dir_path = os.path.join(self.models_dir, "iter_{}".format(self.i))
        os.makedirs(dir_path, exist_ok=True)
        if os.listdir(dir_path):
            return None
        hours = (time.time() - self.start_time) / 3600.0
        self.i += 1
        self.path = os.path.join(dir_path, "model-{}-{}".format(hours, trainer.global_step))
        return save(self.path, trainer, self.with_slots)


class PeriodicPerStepCallback(object):
    """OpenAIGym/common.py:159-170: trigger the wrapped callback every n steps."""

    def __init__(self, cb, n):
        self.cb, self.n, self.counter = cb, int(n), 0

    def trigger_step(self, trainer):
        self.counter += 1
        if self.counter == self.n:
            self.counter = 0
            return self.cb.trigger_step(trainer)
        return None
