"""Fixture-generation shim: the base class ``dataset.py:28`` derives from (never instantiated here)."""


class Dataset:
    pass
