"""CPU checks of the C ABI boundary: libba3c.so loads, exports every function that
include/ba3c.h declares, and its host-only entry points (config validation, flat parameter
layout, workspace sizing) agree with the reference's variable inventory (train.py:177-264).
No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import ba3c_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ba3c.h")


def _lib():
    from ba3c_amd import _lib as L
    return L, L.load()


def test_library_exports_every_header_symbol():
    L, lib = _lib()
    text = open(HEADER).read()
    names = set(re.findall(r"^\s*(?:int|void|const char\*|int64_t|size_t)\s+(ba3c_\w+)\s*\(", text, re.M))
    assert len(names) >= 15, names
    for n in sorted(names):
        assert hasattr(lib, n), "libba3c.so does not export %s" % n
    assert lib.ba3c_version() == 1


def _create(**kw):
    L, lib = _lib()
    cfg = dict(max_batch=32, channels=4, fc_neurons=128, fc_splits=4, num_actions=4,
               replace_with_conv=1, ps=1)
    cfg.update(kw)
    c = L.Ba3cConfig(**cfg)
    h = ctypes.c_void_p()
    st = lib.ba3c_create(ctypes.byref(c), ctypes.byref(h))
    return L, lib, st, h


def _layout(lib, h):
    out = []
    for i in range(lib.ba3c_num_tensors(h)):
        name = ctypes.c_char_p()
        off, numel = ctypes.c_int64(), ctypes.c_int64()
        shape = (ctypes.c_int32 * 4)()
        nd = ctypes.c_int32()
        assert lib.ba3c_tensor_info(h, i, ctypes.byref(name), ctypes.byref(off), ctypes.byref(numel),
                                    shape, ctypes.byref(nd)) == 0
        out.append((name.value.decode(), off.value, numel.value, tuple(shape[k] for k in range(nd.value))))
    return out


@pytest.mark.parametrize("F,S,A,legacy,ps", [(128, 4, 4, False, 1), (512, 1, 6, False, 1),
                                             (256, 1, 18, True, 4)])
def test_layout_matches_reference_inventory(F, S, A, legacy, ps):
    L, lib, st, h = _create(fc_neurons=F, fc_splits=S, num_actions=A,
                            replace_with_conv=0 if legacy else 1, ps=ps)
    assert st == 0, lib.ba3c_last_error()
    lay = _layout(lib, h)
    specs = O.param_specs(F, S, A, replace_with_conv=not legacy, ps=ps)
    assert [(n, s) for n, _, _, s in lay] == [(n, tuple(s)) for n, s in specs]
    prev_end = 0
    for n, off, numel, shape in lay:
        assert off % 64 == 0 and off >= prev_end and numel == int(np.prod(shape))
        prev_end = off + numel
    assert lib.ba3c_flat_size(h) >= prev_end
    ws_t = lib.ba3c_workspace_size(h, 32, 1)
    ws_f = lib.ba3c_workspace_size(h, 32, 0)
    assert ws_t > ws_f > 32 * 84 * 84
    lib.ba3c_destroy(h)


@pytest.mark.parametrize("bad", [dict(channels=3), dict(num_actions=0), dict(num_actions=40),
                                 dict(fc_neurons=130), dict(max_batch=0), dict(fc_splits=3)])
def test_create_rejects_bad_config(bad):
    L, lib, st, h = _create(**bad)
    assert st == 1
    assert len(lib.ba3c_last_error()) > 0


def test_entry_points_reject_null_pointers_without_gpu():
    L, lib, st, h = _create()
    assert st == 0
    r = lib.ba3c_train_grads(h, None, None, None, None, None, 32, 0.01, None, None, None)
    assert r == 1 and b"pointer" in lib.ba3c_last_error()
    r = lib.ba3c_forward(h, None, None, None, 4, 1.0, None, None, None, None)
    assert r == 1
    lib.ba3c_destroy(h)


def test_clip_partials_do_not_alias_activations():
    """The clip / optimizer sum-of-squares partials sit in a batch-independent first region of
    every workspace: no intermediate tensor starts before it ends."""
    L, lib, st, h = _create()
    assert st == 0
    for train in (0, 1):
        for B in (1, 32):
            off, nb = ctypes.c_int64(), ctypes.c_int64()
            assert lib.ba3c_workspace_tensor(h, B, train, b"p0", ctypes.byref(off), ctypes.byref(nb)) == 0
            assert off.value >= 256
    lib.ba3c_destroy(h)


@pytest.mark.parametrize("F,S,legacy,ps,conv_init,fc_init",
                         [(128, 4, False, 1, "normal", "uniform"), (512, 1, False, 1, "xavier", "normal"),
                          (256, 1, True, 4, "uniform", "uniform")])
def test_product_initialisers_match_oracle_restatement(F, S, legacy, ps, conv_init, fc_init):
    """ba3c_amd.initializers (conv2d.py:48-55, fc.py:35-38) draws, for a layout and seed, the
    same values as the oracle's independent restatement."""
    from ba3c_amd.initializers import initial_values
    L, lib, st, h = _create(fc_neurons=F, fc_splits=S, replace_with_conv=0 if legacy else 1, ps=ps)
    lay = _layout(lib, h)
    lib.ba3c_destroy(h)
    got = initial_values(lay, seed=3, conv_init=conv_init, fc_init=fc_init,
                         replace_with_conv=not legacy)
    ref = O.init_params(F, S, 4, seed=3, conv_init=conv_init, fc_init=fc_init,
                        replace_with_conv=not legacy, ps=ps)
    assert list(got) == list(ref)
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k])
    assert np.abs(got["conv1/W"]).max() <= (0.06 if conv_init == "normal" else 0.2)
