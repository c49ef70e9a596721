"""rave_amd -- MI355X-native (gfx950) RAVE encode->decode path.

Python surface of the reference's ``rave.model.RAVE`` (encode / decode /
forward) over hand-written HIP kernels behind a C-ABI (include/rave_amd.h).
Importing the model needs the in-tree native library ``rave_amd/librave_amd.so``;
config / graph / weight utilities are importable without it.
"""
from .config import RaveConfig, get_config  # noqa: F401

__all__ = ["RaveConfig", "get_config", "RAVE"]


def __getattr__(name):
    if name == "RAVE":
        from .model import RAVE
        return RAVE
    if name == "StreamingRAVE":
        from .streaming import StreamingRAVE
        return StreamingRAVE
    raise AttributeError(name)
