"""hgin — MI355X-native (gfx950) heterogeneous-GIN training hot path.

Drop-in for the reference's ``models.py`` surface (HetroGIN / GINLayer / GINConv over a PyG-style
HeteroConv / MessagePassing), with the message + aggregate, the self term, the MLP update (MFMA), their
backward, the CSR build, the negative sampler and the link decoder in hand-written HIP (libhgin.so, C ABI
in include/hgin.h).  See DESIGN.md.
"""
from . import data  # noqa: F401
from ._lib import HginError, HginUnavailable, build  # noqa: F401
from .conv import GINConv, GINLayer, HeteroConv, MessagePassing, reset  # noqa: F401
from .models import HetroGAT, HetroGIN  # noqa: F401
from .qt import QTBaseline  # noqa: F401

__all__ = ["HetroGIN", "HetroGAT", "QTBaseline", "GINLayer", "GINConv", "HeteroConv", "MessagePassing", "reset", "build",
           "HginError", "HginUnavailable", "data"]
