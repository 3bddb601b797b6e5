"""Variable initialisers of the reference graph, for a fresh network in the product package.

Conv2D (tensorpack_cpu/tensorpack/models/conv2d.py:48-55) picks its W initialiser by
`conv_init`:  'normal'  -> tf.truncated_normal_initializer(stddev=3e-2)
              'uniform' -> tf.random_uniform_initializer(-0.05, 0.05)
              'uniform2'-> tf.uniform_unit_scaling_initializer(factor=1.43)   (fc1 convs,
                           OpenAIGym/train.py:221)
              'xavier'  -> tf.contrib.layers.xavier_initializer_conv2d()
FullyConnected (models/fc.py:35-38) by `fc_init`:
              'normal'  -> tf.truncated_normal_initializer(stddev=1/sqrt(in_dim))
              'uniform' -> tf.uniform_unit_scaling_initializer(factor=1.43)
Biases: tf.constant_initializer() = 0.

TF's random streams cannot be reproduced bit for bit (its Philox generator is not in this
image), so the draws come from numpy's RandomState with TF's distributions: a truncated normal
re-draws every sample outside 2 stddev, the unit-scaling bound is factor*sqrt(3/fan_in) with
fan_in = prod(shape[:-1]), and xavier's conv bound is sqrt(6/(fan_in + fan_out)) with the
receptive field counted on both sides.  The draw order is the engine's tensor order (the
reference's variable creation order), one RandomState for the whole network.
"""
import math

import numpy as np


class TruncatedNormal(object):
    def __init__(self, stddev):
        self.stddev = float(stddev)

    def __call__(self, rs, shape):
        out = rs.normal(0.0, self.stddev, size=shape)
        bad = np.abs(out) > 2 * self.stddev
        while bad.any():
            out[bad] = rs.normal(0.0, self.stddev, size=int(bad.sum()))
            bad = np.abs(out) > 2 * self.stddev
        return out


class RandomUniform(object):
    def __init__(self, lo, hi):
        self.lo, self.hi = float(lo), float(hi)

    def __call__(self, rs, shape):
        return rs.uniform(self.lo, self.hi, size=shape)


class UniformUnitScaling(object):
    def __init__(self, factor=1.0):
        self.factor = float(factor)

    def __call__(self, rs, shape):
        fan_in = int(np.prod(shape[:-1]))
        lim = self.factor * math.sqrt(3.0 / fan_in)
        return rs.uniform(-lim, lim, size=shape)


class XavierConv2d(object):
    def __call__(self, rs, shape):
        kh, kw, cin, cout = shape
        lim = math.sqrt(6.0 / (kh * kw * cin + kh * kw * cout))
        return rs.uniform(-lim, lim, size=shape)


def conv_initializer(conv_init):
    """The W initialiser Conv2D builds for `conv_init` (conv2d.py:48-55)."""
    if conv_init == "normal":
        return TruncatedNormal(3e-2)
    if conv_init == "uniform":
        return RandomUniform(-0.05, 0.05)
    if conv_init == "uniform2":
        return UniformUnitScaling(1.43)
    if conv_init == "xavier":
        return XavierConv2d()
    raise ValueError("unknown conv_init %r" % conv_init)


def fc_initializer(fc_init, in_dim):
    """The W initialiser FullyConnected builds for `fc_init` (fc.py:35-38)."""
    if fc_init == "normal":
        return TruncatedNormal(1.0 / math.sqrt(float(in_dim)))
    if fc_init == "uniform":
        return UniformUnitScaling(1.43)
    raise ValueError("unknown fc_init %r" % fc_init)


def initial_values(layout, seed=0, conv_init="normal", fc_init="uniform",
                   replace_with_conv=True, dtype=np.float32):
    """{name: ndarray} for every tensor of an engine layout [(name, offset, numel, shape)].

    conv0..conv3/W: `conv_init` (train.py:177-207); fc1_i/W: 'uniform2' when FC1 is built as
    convs (train.py:216-229), else FullyConnected's `fc_init` (train.py:230-243); fc-pi/W,
    fc-v/W: `fc_init` (train.py:250-259); every bias 0."""
    rs = np.random.RandomState(seed)
    out = {}
    for name, _, _, shape in layout:
        if name.endswith("/b"):
            v = np.zeros(shape)
        elif name.startswith("conv"):
            v = conv_initializer(conv_init)(rs, shape)
        elif name.startswith("fc1_") and replace_with_conv:
            v = conv_initializer("uniform2")(rs, shape)
        else:
            v = fc_initializer(fc_init, shape[0])(rs, shape)
        out[name] = np.asarray(v, dtype=dtype)
    return out
