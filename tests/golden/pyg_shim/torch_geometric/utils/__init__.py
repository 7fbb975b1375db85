def to_dense_adj(*args, **kwargs):  # models.py:170-177 compute_identity is dead code
    raise NotImplementedError("pyg_shim: to_dense_adj is not restated")
