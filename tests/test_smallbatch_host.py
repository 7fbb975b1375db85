"""Host side of the fused small-batch step (hgin/smallbatch.py) on the CPU: the ctypes mirror of the kernels' argument
block against the library's own sizeof / offsetof (no device call), which models it takes, and that a model it does
not take is refused with the reason.  The step itself is tests/test_gpu_smallbatch.py."""
import pytest
import torch

from hgin import HetroGIN
from hgin.data import CONFIGS
from hgin.smallbatch import SmallBatchStep, _structure, check_layout


def _kw(**o):
    # (HetroGIN edits its input_channels dict in place, as the reference does: a fresh one per model)
    return dict(CONFIGS["cfg1"].model_kwargs({"link": 7, "path": 7, "node": 3}), **o)


def test_argument_block_layout_matches_the_library():
    check_layout()


def test_supported_models():
    assert SmallBatchStep.supports(HetroGIN(**_kw()))
    assert SmallBatchStep.supports(HetroGIN(**_kw(message_passing_layers=3)))
    assert SmallBatchStep.supports(HetroGIN(**_kw(mlp_layers=[64, 32, 16])))
    assert SmallBatchStep.supports(HetroGIN(**_kw(global_feats=True, bl_features=True)))
    assert SmallBatchStep.supports(HetroGIN(**_kw(node_embedding_size=128)))
    assert SmallBatchStep.supports(HetroGIN(**_kw(mlp_bn=True, global_feats=True, bl_features=True)))


@pytest.mark.parametrize("override,reason", [
    ({"dropout": 1.0}, "dropout probability"),
    ({"mlp_head_act": "torch.nn.PReLU()"}, "head"),
    ({"node_embedding_size": 256}, "widths"),
    ({"message_passing_layers": 5}, "layers"),
])
def test_refused_models_say_why(override, reason):
    st = _structure(HetroGIN(**_kw(**override)))
    assert isinstance(st, str) and reason in st, st


def test_refuses_a_non_capturable_optimizer_before_touching_the_device():
    """Adam is folded into the step (any capturable setting); another optimizer must be capturable, as must Adam
    when folding is switched off."""
    from hgin.smallbatch import foldable
    model = HetroGIN(**_kw())
    assert foldable(torch.optim.Adam(model.parameters(), lr=1e-3))
    assert not foldable(torch.optim.Adam(model.parameters(), lr=1e-3, amsgrad=True))
    assert not foldable(torch.optim.AdamW(model.parameters(), lr=1e-3))
    #  updates the folded kernel would not reproduce, or parameters it would train against the caller's wish
    if "decoupled_weight_decay" in torch.optim.Adam([torch.zeros(1, requires_grad=True)]).defaults:
        assert not foldable(torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-2,
                                             decoupled_weight_decay=True))
    params = list(model.parameters())
    assert foldable(torch.optim.Adam(params, lr=1e-3, weight_decay=1e-2), params)
    assert not foldable(torch.optim.Adam(params[1:], lr=1e-3), params)          # a parameter left out
    params[0].requires_grad_(False)
    assert not foldable(torch.optim.Adam(params, lr=1e-3), params)              # a frozen parameter
    params[0].requires_grad_(True)
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)   # not capturable
    with pytest.raises(ValueError, match="capturable"):
        SmallBatchStep(model, opt, store=None, batch_size=8, warmup_ids=[[0]])
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)   # capturable=False, folding off
    with pytest.raises(ValueError, match="capturable"):
        SmallBatchStep(model, opt, store=None, batch_size=8, warmup_ids=[[0]], fold_optimizer=False)


def test_fused_eval_takes_the_fused_models():
    from hgin.smallbatch import SmallBatchEval
    assert SmallBatchEval.supports(HetroGIN(**_kw()))
    assert SmallBatchEval.supports(HetroGIN(**_kw(global_feats=True, bl_features=True, dropout=0.2)))
    assert SmallBatchEval.supports(HetroGIN(**_kw(mlp_bn=True)))   # eval-mode BatchNorm: an affine map
    m = HetroGIN(**_kw())
    with pytest.raises(ValueError, match="model.eval"):   # (before any device work)
        SmallBatchEval(m, None, 4, warmup_ids=[[0]])
