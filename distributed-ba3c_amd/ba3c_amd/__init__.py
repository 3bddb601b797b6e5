"""ba3c_amd — MI355X-native BA3C learner/predictor hot path (HIP kernels in libba3c.so)."""
from ._lib import Ba3cLibraryError, LIB_PATH, SCALAR_NAMES, load as load_library  # noqa: F401
from .model_desc import (InputVar, MapGradient, ModelDesc, TowerContext,  # noqa: F401
                         clip_by_average_norm, get_current_tower_context)

__all__ = ["Ba3cEngine", "Model", "Ba3cTrainer", "TrainConfig", "OnlinePredictor",
           "MultiThreadAsyncPredictor", "AdamOptimizer", "RMSPropOptimizer",
           "SyncReplicasOptimizer", "make_optimizer", "InputVar", "ModelDesc", "TowerContext",
           "MapGradient", "clip_by_average_norm", "get_current_tower_context",
           "Ba3cLibraryError", "load_library"]


def __getattr__(name):
    # torch-dependent modules are imported lazily so the C-ABI checks run without a GPU stack
    if name == "Ba3cEngine":
        from .engine import Ba3cEngine
        return Ba3cEngine
    if name == "Model":
        from .model import Model
        return Model
    if name in ("Ba3cTrainer", "TrainConfig"):
        from . import trainer
        return getattr(trainer, name)
    if name in ("OnlinePredictor", "MultiThreadAsyncPredictor"):
        from . import predict
        return getattr(predict, name)
    if name in ("AdamOptimizer", "RMSPropOptimizer", "SyncReplicasOptimizer", "make_optimizer",
                "GradientDescentOptimizer", "MomentumOptimizer", "AdagradOptimizer",
                "AdadeltaOptimizer"):
        from . import optimizer
        return getattr(optimizer, name)
    raise AttributeError(name)
