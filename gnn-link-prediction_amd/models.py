"""Drop-in replacement for the reference's ``models.py`` (youssefshoeb/GNN-Link-Prediction).

Put this directory on ``sys.path`` in place of the reference checkout and ``train.py``'s
``from models import HetroGAT, HetroGIN`` (train.py:8) and ``dataset.py``'s ``from models import QTBaseline``
(dataset.py:13) resolve here unchanged; the GIN path and the queueing-theory baseline run on libhgin.so
(HIP, gfx950).  See INTEGRATION.md.
"""
from hgin.conv import GINConv, GINLayer, HeteroConv, MessagePassing, reset  # noqa: F401
from hgin.models import HetroGAT, HetroGIN  # noqa: F401
from hgin.qt import QTBaseline  # noqa: F401
