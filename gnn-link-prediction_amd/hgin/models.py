"""HetroGIN — drop-in for the reference's ``models.py:248-376`` on the MI355X HIP path.

Constructor keywords, the (mutated) ``input_channels`` dict, parameter initialisation order (and therefore
the values under a given ``torch.manual_seed``), ``state_dict`` keys and ``forward(x_dict,
edge_index_dict, path_batch) -> Tensor[N_path, 1]`` are those of the reference, so ``train.py``'s
``load_model`` (``train.py:116-137``), the training loop (``train.py:16-67``) and ``load_state_dict`` of a
reference checkpoint (``train.py:327``) work unchanged.  Message passing runs on libhgin.so; the readout
MLP and the optional global pooling are small dense torch ops on the device.

``HetroGAT`` (``models.py:380-506``, SURVEY.md §8 F4's second conv family) shares HetroGIN's feature slicing, relation
loop and readout, with the GATConv layers of ``hgin/gat.py``.
"""
from __future__ import annotations

import weakref
from typing import List

import torch

from . import ops
from .conv import GINLayer, HeteroConv, _fusable_mlp as _fusable_linear_prelu

_ACTS = {"torch.nn.PReLU()": torch.nn.PReLU, "torch.nn.ReLU()": torch.nn.ReLU, "torch.nn.ELU()": torch.nn.ELU,
         "torch.nn.LeakyReLU()": torch.nn.LeakyReLU, "torch.nn.Tanh()": torch.nn.Tanh,
         "torch.nn.Sigmoid()": torch.nn.Sigmoid, "torch.nn.GELU()": torch.nn.GELU,
         "torch.nn.SiLU()": torch.nn.SiLU, "torch.nn.Identity()": torch.nn.Identity}


def make_activation(spec):
    """The reference ``eval``s the activation string (models.py:301, :328-330); here a whitelist."""
    if isinstance(spec, torch.nn.Module):
        return spec
    try:
        return _ACTS[spec]()
    except KeyError:
        raise ValueError(f"unsupported activation {spec!r}; expected one of {sorted(_ACTS)}") from None


def _host_call_device(model: torch.nn.Module, x_dict, edge_index_dict, path_batch):
    """The HIP device to run a host-resident call on, or None when inputs and parameters are already on it.

    ``train.py:322-348`` (``evaluate``) builds the model and the batches on the CPU and never calls
    ``.cuda()``; there the call runs on the MI355X (there is no CPU fallback) and the result comes back to
    the CPU.  Without a HIP device it raises."""
    tensors = list(x_dict.values()) + list(edge_index_dict.values()) + [path_batch]
    tensors += [p for p in model.parameters()]
    if all(t is None or t.is_cuda for t in tensors):
        return None
    if any(t is not None and t.is_cuda for t in tensors):
        devs = sorted({str(t.device) for t in tensors if t is not None})
        raise RuntimeError(f"HetroGIN: inputs and parameters on different devices {devs}")
    from ._lib import HginUnavailable
    if not torch.cuda.is_available():
        raise HginUnavailable("HetroGIN: the MI355X path has no CPU fallback and no HIP device is visible")
    return torch.device("cuda", torch.cuda.current_device())


_LENT: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()   # model -> {id(t): (key, dev copy, ref(t), snapshot)}


def release_device_cache(model: torch.nn.Module) -> None:
    """Drop the device copies (and host snapshots) a host-resident model keeps between ``evaluate()`` calls."""
    _LENT.pop(model, None)


def _host_call(model: torch.nn.Module, dev, x_dict, edge_index_dict, path_batch):
    """Run ``model`` on ``dev`` for a host-resident inference call (``evaluate``, train.py:331-335 runs it under
    ``torch.set_grad_enabled(False)``): parameters and buffers are lent to the device for the call and restored
    afterwards (same Parameter objects), inputs are copied over, the output returns to the host.  The host
    copies of the inputs are not modified (PyG's ``x_dict`` is a fresh dict per access).  A gradient-recording
    host call raises: training moves the model to the device first (``model.cuda()``, train.py:177)."""
    if torch.is_grad_enabled() and any(p.requires_grad for p in model.parameters()):
        raise RuntimeError("HetroGIN: a host-resident call with gradients enabled; move the model to the HIP "
                           "device for training (model.cuda(), train.py:177) or call it under torch.no_grad() / "
                           "torch.set_grad_enabled(False) as train.py's evaluate() does")
    host = next(iter(x_dict.values())).device
    lent = []
    seen = set()
    for t in list(model.parameters()) + list(model.buffers()):
        if id(t) not in seen:
            seen.add(id(t))
            lent.append((t, t.data))
    # device copies are kept per model between calls (evaluate() runs one call per batch with unchanged weights) and
    # re-copied when a tensor's version, storage, shape or VALUES changed: load_state_dict, in-place edits, and edits
    # through ``p.data`` (which do not bump ``p._version``) — each call compares the host tensor with a host snapshot
    # taken when its copy was made (O(parameters) on the host; no device traffic).  The cache holds a device copy and a
    # host snapshot of every parameter and buffer while the model lives: release_device_cache(model) drops them.
    cache = _LENT.setdefault(model, {})
    try:
        for t, d in lent:
            key = (t._version, d.data_ptr(), tuple(d.shape), d.dtype, str(dev))
            hit = cache.get(id(t))
            if hit is None or hit[0] != key or hit[2]() is not t or not torch.equal(d, hit[3]):
                hit = (key, d.to(dev), weakref.ref(t), d.clone())
                cache[id(t)] = hit
            t.data = hit[1]
        xd = {k: v.to(dev) for k, v in x_dict.items()}
        ed = {k: v.to(dev) for k, v in edge_index_dict.items()}
        pb = path_batch.to(dev) if path_batch is not None else None
        out = model._run(xd, ed, pb, None, None)
        res = out.to(host)   # (this call syncs the host anyway: an unsorted GLOBAL_FEATS batch vector raises here)
        if getattr(model, "global_feats", False):
            ops.check_pool_order()
    finally:
        for t, d in lent:
            t.data = d
    return res


class HetroGIN(torch.nn.Module):
    """models.py:248-376 on the MI355X path (module docstring).  With ``global_feats`` the path batch vector must be
    non-decreasing, as PyG's collation makes it (and GraphStore's batches are by construction): the pooling kernel
    flags a descending pair in a device status word instead of syncing the host every step — the host-resident
    ``evaluate()`` call checks it (and raises), a training step leaves it to ``ops.check_pool_order()``; an unsorted
    vector otherwise yields unspecified pooled features."""

    def __init__(self, input_channels: dict, node_embedding_size: int, message_passing_layers: int, dropout: float,
                 concat_path: bool, bl_features: bool, divided_features: bool, global_feats: bool,
                 mlp_layers: list, act, mlp_head_act, mlp_bn: bool):
        super().__init__()
        self.num_layers = message_passing_layers
        self.concat_path = concat_path
        self.bl_features = bl_features
        self.divided_features = divided_features
        self.mlp_layers = mlp_layers
        self.dropout = dropout
        self.global_feats = global_feats

        # models.py:260-269 (mutates the caller's dict, as the reference does)
        if not self.divided_features:
            input_channels["path"] = input_channels["path"] - 3
            input_channels["link"] = input_channels["link"] - 1
            if not self.bl_features:
                input_channels["path"] = input_channels["path"] - 1
                input_channels["link"] = input_channels["link"] - 3
        else:
            if not self.bl_features:
                input_channels["path"] = input_channels["path"] - 1
                input_channels["link"] = input_channels["link"] - 3

        self.global_feats_size = 8 if global_feats else 0
        self.concat_size = input_channels["path"] if concat_path else 0

        self.convs = torch.nn.ModuleList()
        self.readout = torch.nn.ModuleList()
        ic, H = input_channels, node_embedding_size
        # models.py:286-290 first conv layer (concat self term)
        self.convs.append(HeteroConv({
            ("path", "uses", "link"): GINLayer(ic["path"] + ic["link"], H, concat=True),
            ("link", "includes", "path"): GINLayer(ic["link"] + ic["path"], H, concat=True),
            ("link", "connects", "node"): GINLayer(ic["link"] + ic["node"], H, concat=True),
            ("node", "has", "link"): GINLayer(ic["node"] + ic["link"], H, concat=True)}, aggr="sum"))
        # models.py:293-298 remaining conv layers (add self term)
        for _ in range(self.num_layers - 1):
            self.convs.append(HeteroConv({
                ("path", "uses", "link"): GINLayer(H, H),
                ("link", "includes", "path"): GINLayer(H, H),
                ("link", "connects", "node"): GINLayer(H, H),
                ("node", "has", "link"): GINLayer(H, H)}, aggr="sum"))

        # models.py:301-330 readout (ONE activation instance shared by the hidden readout layers)
        act = make_activation(act)
        width0 = H + self.concat_size + self.global_feats_size
        for i in range(len(mlp_layers)):
            lin = torch.nn.Linear(width0 if i == 0 else mlp_layers[i - 1], mlp_layers[i])
            if mlp_bn:
                self.readout.append(torch.nn.Sequential(lin, torch.nn.BatchNorm1d(num_features=mlp_layers[i]), act))
            else:
                self.readout.append(torch.nn.Sequential(lin, act))
        if mlp_head_act is None:
            self.readout.append(torch.nn.Sequential(torch.nn.Linear(mlp_layers[-1], 1)))
        else:
            self.readout.append(torch.nn.Sequential(torch.nn.Linear(mlp_layers[-1], 1),
                                                    make_activation(mlp_head_act)))

    def prune_dead(self, enable: bool = True) -> List[str]:
        """Skip relations whose outputs cannot reach the readout.  Off by default: the
        reference computes every relation in every layer; pruned runs are reported separately."""
        dead: List[str] = []
        live_types = {"path"}
        for li in range(self.num_layers - 1, -1, -1):
            conv = self.convs[li]
            conv.skip = set()
            needed = set()
            for key in conv.convs.keys():
                src, _, dst = key.split("__")
                if dst in live_types:
                    needed.add(src)
                    needed.add(dst)
                elif enable:
                    conv.skip.add(key)
                    dead.append(f"{li}:{key}")
            live_types = needed
        return dead

    def forward(self, x_dict, edge_index_dict, path_batch):
        dev = _host_call_device(self, x_dict, edge_index_dict, path_batch)
        if dev is not None:
            return _host_call(self, dev, x_dict, edge_index_dict, path_batch)
        return self._run(x_dict, edge_index_dict, path_batch, None, None)

    def forward_loss(self, x_dict, edge_index_dict, path_batch, y, m_valid=None):
        """(out, loss_value) with loss_value = train.py's mape(out, y.reshape(-1, 1)) (train.py:12-13, :38-40).

        When the head is the plain Linear(mlp_layers[-1], 1) (mlp_head_act None, the reference default), the
        head and the loss run as one fused pass forward and one backward (ops.head_mape):
        no per-element torch kernels and no host sync; ``out`` carries no gradient.  Otherwise the head
        runs as usual and the loss is the torch expression.  ``m_valid`` (device int32 [1], fused head only):
        the loss covers path rows < m_valid (padded static-shape batches, hgin/graphs.py)."""
        return self._run(x_dict, edge_index_dict, path_batch, y, m_valid)

    def _run(self, x_dict, edge_index_dict, path_batch, y, m_valid):
        self._select_features(x_dict)
        origin_input = x_dict.copy()

        pooled = None
        if self.global_feats:   # models.py:347-352: [mean | max] per graph, gathered to the rows, in one launch
            pooled = ops.global_pool(origin_input["path"], path_batch)

        for i in range(self.num_layers):   # models.py:355-359
            x_dict = self.convs[i](x_dict, edge_index_dict)
            if self.dropout > 0.0 and self.training:
                for k in list(x_dict.keys()):
                    x_dict[k] = torch.nn.functional.dropout(x_dict[k], p=self.dropout, training=True)
        return self._readout(x_dict["path"], origin_input["path"], pooled, y, m_valid)

    def _select_features(self, x_dict):
        """models.py:333-342 feature slicing (assigns into the caller's dict, as the reference does)."""
        if not self.divided_features:
            x_dict["path"] = torch.cat([x_dict["path"][:, 0:3], x_dict["path"][:, 6].reshape(-1, 1)], axis=1)
            x_dict["link"] = torch.cat([x_dict["link"][:, 0:3], x_dict["link"][:, 4:7]], axis=1)
            if not self.bl_features:
                x_dict["path"] = x_dict["path"][:, 0:3]
                x_dict["link"] = x_dict["link"][:, 0:3]
        else:
            if not self.bl_features:
                x_dict["path"] = x_dict["path"][:, 0:6]
                x_dict["link"] = x_dict["link"][:, 0:3]

    def _readout(self, x_path, origin_path, pooled, y, m_valid):
        """models.py:362-376 on the final path embeddings (+ F3's fused head + loss when ``y`` is given);
        ``pooled`` = [mean | max] global features per row (GLOBAL_FEATS) or None."""
        x2 = None   # second column block of the readout input, read in place instead of torch.cat
        if self.concat_path:   # models.py:362-371
            if pooled is not None:
                x = torch.cat((x_path, origin_path, pooled), 1)
            else:
                x, x2 = x_path, origin_path
        else:
            if pooled is not None:
                x = torch.cat((x_path, pooled), 1)
            else:
                x = x_path

        n_ro = len(self.mlp_layers) + 1
        for i in range(n_ro):   # models.py:373-374
            seq = self.readout[i]
            if (y is not None and i == n_ro - 1 and x2 is None and len(seq) == 1
                    and isinstance(seq[0], torch.nn.Linear) and seq[0].bias is not None
                    and seq[0].out_features == 1):
                return ops.head_mape(x, seq[0].weight, seq[0].bias, y, m_valid)   # F3: head + mape fused
            if _fusable_linear_prelu(seq):
                x = ops.linear_prelu(x, seq[0].weight, seq[0].bias, seq[1].weight, x2=x2)
            elif len(seq) == 1 and isinstance(seq[0], torch.nn.Linear) and seq[0].bias is not None:
                x = ops.linear_prelu(x, seq[0].weight, seq[0].bias, None, x2=x2)
            else:
                if x2 is not None:
                    x = torch.cat((x, x2), 1)
                if m_valid is not None and self.training and any(isinstance(m, torch.nn.BatchNorm1d) for m in seq):
                    for mod in seq:   # a padded batch: MLP_BN's statistics over its first m_valid rows only
                        x = _masked_batch_norm(x, mod, m_valid) if isinstance(mod, torch.nn.BatchNorm1d) else mod(x)
                else:
                    x = seq(x)
            x2 = None
        if y is not None:   # head with an activation / mlp_layers == []: unfused loss (train.py:12-13)
            if m_valid is not None:
                raise NotImplementedError("m_valid (padded batches) needs the fused Linear(k, 1) head")
            from .train import mape
            return x, mape(x, y.reshape(-1, 1))
        return x


def _masked_batch_norm(x: torch.Tensor, bn: torch.nn.BatchNorm1d, m_valid: torch.Tensor) -> torch.Tensor:
    """BatchNorm1d in training mode (models.py:303-313, MLP_BN) over the first m_valid rows of a padded batch
    (hgin/graphs.py): those rows' mean and biased variance normalise every row (the padding rows' outputs feed only
    masked loss rows), and the running statistics take the unbiased variance with the layer's momentum — torch's
    BatchNorm on the exact batch, up to the order of the fp32 sums.  m_valid is a device count: no host sync, so
    the step stays capturable.  Padding rows are selected out (not multiplied by 0), so an inf / NaN there cannot
    reach the statistics.  A batch of one valid row (torch raises: "Expected more than 1 value per channel") leaves
    the running statistics and num_batches_tracked unchanged, as the fused step's k_sb_bn does."""
    if bn.momentum is None:
        raise NotImplementedError("masked BatchNorm: momentum=None (cumulative average) is not supported")
    n = x.shape[0]
    mask = (torch.arange(n, device=x.device) < m_valid.to(torch.int64)).unsqueeze(1)
    m = m_valid.to(x.dtype)
    zero = x.new_zeros(())
    mean = torch.where(mask, x, zero).sum(0) / m
    d = torch.where(mask, x - mean, zero)
    var = (d * d).sum(0) / m
    if bn.track_running_stats:
        with torch.no_grad():
            upd = m > 1.0
            rm = bn.running_mean * (1.0 - bn.momentum) + mean.detach() * bn.momentum
            rv = bn.running_var * (1.0 - bn.momentum) + var.detach() * (m / torch.clamp(m - 1.0, min=1.0)) * bn.momentum
            bn.running_mean.copy_(torch.where(upd, rm, bn.running_mean))
            bn.running_var.copy_(torch.where(upd, rv, bn.running_var))
            bn.num_batches_tracked.add_(upd.to(bn.num_batches_tracked.dtype).reshape(bn.num_batches_tracked.shape))
    y = (x - mean) / torch.sqrt(var + bn.eps)
    if bn.affine:
        y = y * bn.weight + bn.bias
    return y


class HetroGAT(HetroGIN):
    """models.py:380-506 (built by train.py:120-125 when config["MODEL"] == "GAT"): the same feature slicing,
    HeteroConv relation loop and readout as HetroGIN, with PyG 2.0.2 GATConv layers (hgin/gat.py: HIP edge
    softmax + weighted aggregate on the relation's CSR / CSC, projections on the MFMA GEMMs).  As in the reference:
    ``input_channels`` is read, not mutated; the first layer is ``GATConv((-1, -1), H, heads=heads, concat=True)``
    (lazy input projections, materialised at the first forward), later layers ``GATConv(H, H)`` — which cannot
    take the first layer's H * heads outputs, so the reference (and this drop-in) runs only with one layer when
    heads > 1; the readout's first Linear takes H * heads + concat_size + global_feats_size columns."""

    def __init__(self, input_channels: dict, node_embedding_size: int, message_passing_layers: int, dropout: float,
                 heads: int, concat_path: bool, bl_features: bool, divided_features: bool, global_feats: bool,
                 mlp_layers: list, act, mlp_head_act, mlp_bn: bool):
        torch.nn.Module.__init__(self)
        from .gat import GATConv
        self.num_layers = message_passing_layers
        self.dropout = dropout
        self.concat_path = concat_path
        self.mlp_layers = mlp_layers
        self.global_feats = global_feats
        self.heads = heads
        self.bl_features = bl_features
        self.divided_features = divided_features
        self.global_feats_size = 8 if global_feats else 0
        if concat_path:   # models.py:396-405: the width of the sliced path features
            if divided_features and bl_features:
                self.concat_size = input_channels["path"]
            elif divided_features:
                self.concat_size = input_channels["path"] - 1
            elif bl_features:
                self.concat_size = input_channels["path"] - 3
            else:
                self.concat_size = input_channels["path"] - 4
        else:
            self.concat_size = 0
        self.convs = torch.nn.ModuleList()
        self.readout = torch.nn.ModuleList()
        H = node_embedding_size
        rels = (("path", "uses", "link"), ("link", "includes", "path"), ("link", "connects", "node"),
                ("node", "has", "link"))
        # models.py:413-418 first layer; :421-426 remaining layers
        self.convs.append(HeteroConv({r: GATConv((-1, -1), H, heads=heads, concat=True) for r in rels}, aggr="sum"))
        for _ in range(self.num_layers - 1):
            self.convs.append(HeteroConv({r: GATConv(H, H) for r in rels}, aggr="sum"))
        # models.py:429-459 readout
        act = make_activation(act)
        width0 = H * heads + self.concat_size + self.global_feats_size
        for i in range(len(mlp_layers)):
            lin = torch.nn.Linear(width0 if i == 0 else mlp_layers[i - 1], mlp_layers[i])
            if mlp_bn:
                self.readout.append(torch.nn.Sequential(lin, torch.nn.BatchNorm1d(num_features=mlp_layers[i]), act))
            else:
                self.readout.append(torch.nn.Sequential(lin, act))
        if mlp_head_act is None:
            self.readout.append(torch.nn.Sequential(torch.nn.Linear(mlp_layers[-1], 1)))
        else:
            self.readout.append(torch.nn.Sequential(torch.nn.Linear(mlp_layers[-1], 1),
                                                    make_activation(mlp_head_act)))

    def prune_dead(self, enable: bool = True):
        raise NotImplementedError("HetroGAT: dead-relation pruning is a HetroGIN benchmark option")
