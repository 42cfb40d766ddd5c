"""A3C around the gfx950 env (nevertiree/Rein48 algorithm/a3c/a3c.py), batched and synchronous."""
from .losses import chunk_loss, segment_stats  # noqa: F401
from .nets import ActorCriticCNN, ActorCriticMLP, make_net  # noqa: F401
from .optim import FlatParams, RMSPropTF1  # noqa: F401
from .trainer import A3CConfig, A3CTrainer  # noqa: F401
