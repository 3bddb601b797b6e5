"""tensorpack ModelDesc / InputVar / TowerContext / MapGradient surface
(tensorpack_cpu/tensorpack/models/model_desc.py:18-156, tfutils/gradproc.py:34-67), kept so
code written against the reference's graph-building API drops in.  "Graph building" here
binds the concrete input tensors to the fused HIP forward(+backward) of libba3c."""
from collections import namedtuple

InputVar = namedtuple("InputVar", ["type", "shape", "name"])   # model_desc.py:18

_CurrentTowerContext = None


class TowerContext(object):
    """model_desc.py:22-90 — 'towerp*' towers are prediction towers (is_training False)."""

    def __init__(self, tower_name, is_training=None):
        self._name = tower_name
        if is_training is None:
            is_training = not self._name.startswith("towerp")
        self._is_training = is_training

    @property
    def is_training(self):
        return self._is_training

    @property
    def is_main_training_tower(self):
        return self.is_training and self._name in ("", "tower0")

    @property
    def name(self):
        return self._name

    def __enter__(self):
        global _CurrentTowerContext
        assert _CurrentTowerContext is None, "Nesting TowerContext!"
        _CurrentTowerContext = self
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        global _CurrentTowerContext
        _CurrentTowerContext = None
        return False


def get_current_tower_context():
    return _CurrentTowerContext


class ModelDesc(object):
    """model_desc.py:92-156."""

    def get_input_vars_desc(self):
        return self._get_input_vars()

    def _get_input_vars(self):
        raise NotImplementedError

    def build_graph(self, model_inputs):
        self._build_graph(model_inputs)

    def _build_graph(self, inputs):
        raise NotImplementedError

    def get_cost(self):
        return self._get_cost()

    def _get_cost(self, *args):
        return self.cost

    def get_gradient_processor(self):
        return []


class GradientProcessor(object):
    def process(self, engine):
        raise NotImplementedError


class ClipByAverageNorm(object):
    """The function object `lambda grad: tf.clip_by_average_norm(grad, clip_norm)` —
    recognised by MapGradient and executed by the fused HIP clip kernel."""

    def __init__(self, clip_norm=0.1):
        if abs(clip_norm - 0.1) > 0:
            raise NotImplementedError("libba3c's fused clip implements clip_norm=0.1 (train.py:330)")
        self.clip_norm = clip_norm


def clip_by_average_norm(clip_norm=0.1):
    return ClipByAverageNorm(clip_norm)


class MapGradient(GradientProcessor):
    """gradproc.py:34-67: apply `func` to every gradient whose variable name matches regex.
    ClipByAverageNorm over '.*' runs as one HIP kernel over the flat gradient buffer; any
    other callable is applied per tensor to the torch views of the device gradients."""

    def __init__(self, func, regex=".*"):
        import re
        self.func = func
        self.regex = regex if regex.endswith("$") else regex + "$"
        self._re = re.compile(self.regex)

    def process(self, engine):
        if isinstance(self.func, ClipByAverageNorm) and self.regex == ".*$":
            engine.clip_grads()
            return
        for name in engine.tensor_names:
            if self._re.match(name.rsplit("/", 1)[0] + "/" + name.rsplit("/", 1)[1]):
                g = engine.view(engine.grads, name)
                if isinstance(self.func, ClipByAverageNorm):
                    raise NotImplementedError("regex-restricted clip not fused")
                out = self.func(g)
                if out is not None and out is not g:
                    g.copy_(out)
