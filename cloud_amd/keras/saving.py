"""Model save / load (directory format, strategy-agnostic).

``<path>/``
    ``cloud_amd_model.json`` -- format marker, class, config (Sequential) and the
                              compile configuration;
    ``weights.pt``          -- ``state_dict`` (plain tensors: loadable with
                              ``torch.load(weights_only=True)``);
    ``model.pkl``           -- cloudpickled architecture for functional / subclassed
                              models (written by this framework only);
    ``optimizer.pt``        -- fused-optimizer state (master weights + moments).

Weights saved under any strategy load under any other (all replicas hold the
same weights; the chief writes) -- reference ``save_and_load.py:89-125``.
"""
from __future__ import annotations

import json
import os

import torch

FORMAT = "cloud_amd.keras/1"


def chief_only(write):
    """Run ``write()`` on the chief (rank 0) only, then barrier so every replica can
    read what was written (all replicas hold identical weights under DP)."""
    import torch.distributed as dist

    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if not multi or dist.get_rank() == 0:
        write()
    if multi:
        dist.barrier()


def save_model(model, path, include_optimizer=True):
    chief_only(lambda: _save_model(model, path, include_optimizer))


def _save_model(model, path, include_optimizer=True):
    os.makedirs(path, exist_ok=True)
    meta = {"format": FORMAT, "class_name": type(model).__name__, "name": model.name}
    from .models import Sequential

    if isinstance(model, Sequential):
        try:
            meta["config"] = model.get_config()
        except Exception:  # pragma: no cover
            meta["config"] = None
    if getattr(model, "optimizer", None) is not None:
        meta["optimizer"] = {"class_name": type(model.optimizer).__name__, "config": model.optimizer.get_config()}
        lossname = getattr(model.loss, "name", None)
        meta["loss"] = {"class_name": type(model.loss).__name__ if model.loss is not None else None,
                        "from_logits": getattr(model.loss, "from_logits", None), "name": lossname}
        meta["metrics"] = [m.name for m in model.compiled_metrics]
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    torch.save(sd, os.path.join(path, "weights.pt"))
    if meta.get("config") is None:
        import cloudpickle

        was = next((p.device for p in model.parameters()), torch.device("cpu"))
        opt, strat_, red = model.optimizer, model._strategy, model._reducer
        model.optimizer, model._strategy, model._reducer = None, None, None
        try:
            model.to("cpu")
            with open(os.path.join(path, "model.pkl"), "wb") as f:
                cloudpickle.dump(model, f)
        finally:
            model.to(was)
            model.optimizer, model._strategy, model._reducer = opt, strat_, red
    if include_optimizer and getattr(model, "optimizer", None) is not None and model.optimizer.impl is not None:
        torch.save(model.optimizer.impl.state_dict(), os.path.join(path, "optimizer.pt"))
    with open(os.path.join(path, "cloud_amd_model.json"), "w") as f:
        json.dump(meta, f, indent=2, default=str)


def load_model(path, compile=True):
    with open(os.path.join(path, "cloud_amd_model.json")) as f:
        meta = json.load(f)
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path} is not a cloud_amd saved model")
    if meta.get("config") is not None:
        from .models import Sequential

        model = Sequential.from_config(meta["config"])
    else:
        import pickle

        with open(os.path.join(path, "model.pkl"), "rb") as f:
            model = pickle.load(f)
    sd = torch.load(os.path.join(path, "weights.pt"), map_location="cpu", weights_only=True)
    own = model.state_dict()
    with torch.no_grad():
        for k, v in sd.items():
            if k in own:
                own[k].copy_(v.to(own[k].dtype))
    if compile and meta.get("optimizer"):
        from . import losses, optimizers

        ocfg = dict(meta["optimizer"]["config"])
        ocfg.pop("name", None)
        lr = ocfg.pop("learning_rate", None)
        cls = getattr(optimizers, meta["optimizer"]["class_name"])
        opt = cls(learning_rate=lr if lr is not None else 1e-3, **ocfg)
        lmeta = meta.get("loss") or {}
        loss = None
        if lmeta.get("class_name"):
            lcls = getattr(losses, lmeta["class_name"])
            loss = lcls(from_logits=lmeta["from_logits"]) if lmeta.get("from_logits") is not None else lcls()
        model.compile(optimizer=opt, loss=loss, metrics=meta.get("metrics") or None)
        model._pending_optimizer_state = os.path.join(path, "optimizer.pt")
    return model
