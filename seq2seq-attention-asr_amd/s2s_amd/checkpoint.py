"""Checkpoints: the reference saves its whole model table with torch.save
(model.t7, model_best_valid_*.t7; timit/timit.lua:551-562) -- the autoencoder's flat parameters
(getParameters, timit.lua:172) plus optimState.  Here: one safetensors file (no code executed on
load) holding every parameter of the flat layout under its module name, the optimizer state
(optim.adadelta paramVariance / accDelta) when given, and the model config + trainer metadata as JSON.
"""
import dataclasses
import json
import math

import torch
from safetensors import safe_open
from safetensors.torch import save_file

from .model import ModelConfig, param_shapes


def save_flat(path, cfg: ModelConfig, params, optim_state=None, meta=None):
    """params: the flat (n,) float32 buffer; optim_state: the Adadelta state bytes (or None)."""
    shapes = param_shapes(cfg)
    n = sum(math.prod(s) for _, s in shapes)
    if params.numel() != n:
        raise ValueError(f"params has {params.numel()} elements, the layout {n}")
    flat = params.detach().to("cpu", torch.float32).contiguous()
    tensors, off = {}, 0
    for name, shp in shapes:
        sz = math.prod(shp)
        tensors[f"param.{name}"] = flat[off:off + sz].view(shp).clone()
        off += sz
    if optim_state is not None:
        tensors["optim.state"] = optim_state.detach().to("cpu").contiguous().view(torch.uint8).clone()
    header = {"format": "s2s_amd-checkpoint-1", "config": json.dumps(dataclasses.asdict(cfg)),
              "meta": json.dumps(meta or {})}
    save_file(tensors, path, metadata=header)


def load_flat(path):
    """-> (cfg, params (n,) float32 CPU, optim_state uint8 CPU or None, meta dict)."""
    with safe_open(path, framework="pt") as f:
        md = f.metadata() or {}
        if md.get("format") != "s2s_amd-checkpoint-1":
            raise ValueError(f"{path}: not an s2s_amd checkpoint")
        cfg = ModelConfig(**json.loads(md["config"]))
        parts = [f.get_tensor(f"param.{name}").reshape(-1) for name, _ in param_shapes(cfg)]
        state = f.get_tensor("optim.state") if "optim.state" in f.keys() else None
        meta = json.loads(md.get("meta", "{}"))
    return cfg, torch.cat(parts), state, meta


def save(path, model, optimizer=None, meta=None):
    """torch.save(paths.concat(savedir, 'model.t7'), model) for a ChorowskiBaseline (+ its Adadelta).
    The step counter and the user seed travel in the metadata, so a resumed run continues the dropout
    mask sequence instead of replaying it from step 1.  The per-rank seed base is NOT saved: every
    data-parallel rank loads the same file and re-derives its own base from (seed, rank)."""
    meta = dict(meta or {})
    meta.setdefault("steps", int(getattr(model, "_steps", 0)))
    meta.setdefault("seed", str(int(getattr(model, "seed", 0))))
    save_flat(path, model.cfg, model.params, optimizer.state if optimizer is not None else None, meta)


def seed_base_for(meta, rank, default):
    """The loading rank's dropout seed base: _mix64(user seed, rank), so replicas resumed from one file keep
    drawing independent nn.Dropout masks (the base mixes in the rank, model.py).  A checkpoint without the
    user seed but with the saved base of an older writer (meta['dropout_seed_base'], rank 0's base) resumes
    rank 0 from that base, with a warning -- its mask sequence continues -- and every other rank from
    _mix64(base, rank), so the replicas still draw independent masks.  A checkpoint with neither
    leaves `default` (the model's own base) in place, also with a warning."""
    import warnings

    from .model import _mix64
    if "seed" in meta:
        return _mix64(int(meta["seed"]), int(rank))
    if "dropout_seed_base" in meta:
        warnings.warn("checkpoint has no user seed (older format): rank 0 resumes from its saved dropout seed "
                      "base, the other ranks from that base mixed with their rank")
        base = int(meta["dropout_seed_base"])
        return base if int(rank) == 0 else _mix64(base, int(rank))
    warnings.warn("checkpoint has no dropout seed: the resumed run draws a new nn.Dropout mask sequence")
    return default


def load(path, model=None, optimizer=None):
    """Restore into an existing model (and optimizer) or build a new ChorowskiBaseline; returns
    (model, meta)."""
    cfg, params, state, meta = load_flat(path)
    if model is None:
        from .model import ChorowskiBaseline
        model = ChorowskiBaseline(cfg)
    elif dataclasses.asdict(model.cfg) != dataclasses.asdict(cfg):
        raise ValueError("checkpoint config differs from the model's")
    model.params.copy_(params.to(model.params.device))
    if "steps" in meta:
        model._steps = int(meta["steps"])
    from .model import _dist_rank
    if "seed" in meta:
        model.seed = int(meta["seed"])
    model.dropout_seed_base = seed_base_for(meta, _dist_rank(), model.dropout_seed_base)
    if optimizer is not None:
        if state is None or state.numel() != optimizer.state.numel():
            raise ValueError("checkpoint holds no matching optimizer state")
        optimizer.state.copy_(state.to(optimizer.state.device))
    return model, meta
