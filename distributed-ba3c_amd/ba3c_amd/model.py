"""The BA3C `Model(ModelDesc)` of OpenAIGym/train.py:138-330, bound to libba3c.

Same method names and input contract as the reference: `_get_input_vars` (train.py:144-151),
`_build_graph(inputs)` (train.py:274-327; is_training=False stops after the predictor
outputs, :302-304), `get_cost`, `get_gradient_processor` (train.py:329-330) and
`vars_for_save` (checkpoint keys).  `_build_graph` executes the fused HIP forward (+ loss
+ backward when training) on the current stream; the results are device tensors.
"""
import numpy as np
import torch

from . import _lib
from .engine import Ba3cEngine
from .model_desc import (InputVar, MapGradient, ModelDesc, clip_by_average_norm,
                         get_current_tower_context)

IMAGE_SIZE = (84, 84)     # train.py:92
FRAME_HISTORY = 4         # train.py:93
LOCAL_TIME_MAX = 5        # train.py:102
GAMMA = 0.99              # train.py:94


class Model(ModelDesc):
    def __init__(self, num_actions, channels=1, fc_neurons=512, fc_splits=1,
                 replace_with_conv=True, ps=1, batch_size=128, max_batch=None, engine=None,
                 seed=0, conv_init="normal", fc_init="uniform"):
        """channels: the reference's --channels (frames per history step; CHANNEL =
        FRAME_HISTORY*channels, train.py:95).  BASELINE's 84x84x4 input is channels=1.
        A new engine starts from the reference initialisers (--conv_init / --fc_init,
        initializers.py) drawn with `seed`; a caller-supplied engine keeps its variables."""
        self.num_actions = num_actions
        self.channel = FRAME_HISTORY * channels
        self.batch_size = batch_size
        if engine is None:
            engine = Ba3cEngine(num_actions=num_actions, channels=self.channel,
                                fc_neurons=fc_neurons, fc_splits=fc_splits,
                                replace_with_conv=replace_with_conv, ps=ps,
                                max_batch=max_batch or max(batch_size, 16))
            engine.init_params(seed=seed, conv_init=conv_init, fc_init=fc_init)
        self.engine = engine
        self.entropy_beta = 0.01      # non-trainable var 'entropy_beta' (train.py:296-297)
        self.explore_factor = 1.0     # non-trainable var 'explore_factor' (train.py:294-295)
        self.vars_for_save = {n: n for n in self.engine.tensor_names}
        self.cost = None

    def _get_input_vars(self):
        return [InputVar(torch.uint8, (None,) + IMAGE_SIZE + (self.channel,), "state"),
                InputVar(torch.int64, (None,), "action"),
                InputVar(torch.float32, (None,), "futurereward"),
                InputVar(torch.float32, (self.batch_size,), "global_step_from_predict"),
                InputVar(torch.float32, (None,), "init_R"),
                InputVar(torch.bool, (None,), "isOver")]

    def _build_graph(self, inputs):
        state, action, futurereward = inputs[0], inputs[1], inputs[2]
        ctx = get_current_tower_context()
        is_training = True if ctx is None else ctx.is_training
        if not is_training:
            self.logits, self.logitsT, self.value = self.engine.forward(
                state, explore_factor=self.explore_factor)
            return
        self.delay = inputs[3] if len(inputs) > 3 else None
        # train_phase 1 / 2: the two halves of the pass around the fc1 + heads gradient bucket
        # (Ba3cTrainer's bucketed data-parallel step); 0: the whole pass
        sc = self.engine.train_grads(state, action, futurereward, entropy_beta=self.entropy_beta,
                                     phase=getattr(self, "train_phase", 0))
        self.scalars = sc
        self.cost = sc[0]

    def get_gradient_processor(self):
        return [MapGradient(clip_by_average_norm(0.1))]

    def get_predict_func(self, input_names=("state",), output_names=("logitsT", "pred_value")):
        from .predict import OnlinePredictor
        return OnlinePredictor(self, input_names, output_names)

    def scalars_dict(self):
        vals = self.scalars.tolist()
        d = dict(zip(_lib.SCALAR_NAMES, vals))
        d["active_relus"] = int(round(d["active_relus"]))
        return d
