"""Fixture-generation shim for PyG 2.0.2 (see ../README.md). Not the product; not the oracle."""
__version__ = "2.0.2-shim"
from . import typing  # noqa: F401
from . import utils  # noqa: F401
from . import nn  # noqa: F401
from . import data  # noqa: F401
