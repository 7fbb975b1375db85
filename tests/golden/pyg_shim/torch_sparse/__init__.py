class SparseTensor:  # models.py:222-225 message_and_aggregate is unreachable with [2,E] edge_index
    def __init__(self, *a, **k):
        raise NotImplementedError("pyg_shim: SparseTensor is not restated")


def matmul(*a, **k):
    raise NotImplementedError("pyg_shim: torch_sparse.matmul is not restated")
