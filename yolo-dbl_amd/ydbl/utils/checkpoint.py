"""Reference ``.pt`` checkpoints, read without executing anything from the file.

The reference trainer saves ``torch.save({"ema": <fp16 DetectionModel object>, "model": None,
"train_args": {...}, "date": ..., ...})`` (U/engine/trainer.py:513-546) and loads it back with a
full unpickler (torch_safe_load / attempt_load_one_weight, U/nn/tasks.py:804-944).  Here the file is
read with torch's weights-only unpickler: every class the pickle names under an allowed family
(``ultralytics.*``, ``torch.nn.modules.*``, numpy scalars/dtypes, SimpleNamespace) is bound to an inert
placeholder that only records its constructor arguments and state, so no code from the file runs.
Any other global is refused.  The placeholder tree is then walked like nn.Module.state_dict()
(parameters, persistent buffers, submodules), cast to fp32 as attempt_load_one_weight does, and
paired with the model's embedded ``yaml`` dict and ``names``.
"""

from __future__ import annotations

from pathlib import Path

import torch

ALLOWED_PREFIXES = ("ultralytics.", "torch.nn.modules.", "torch.nn.functional.", "numpy.", "types.SimpleNamespace", "argparse.Namespace",
                    "pathlib.", "collections.", "builtins.set", "builtins.frozenset", "__builtin__.set")


class _Inert:
    """Placeholder for a pickled object: keeps constructor args and __setstate__ state, runs nothing."""

    def __init__(self, *args, **kwargs):
        self.__dict__["_args"] = args

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2 and isinstance(state[0], (dict, type(None))):
            state, slots = state  # (dict state, slot state) form
            if isinstance(slots, dict):
                self.__dict__.update(slots)
        if isinstance(state, dict):
            self.__dict__.update(state)
        else:
            self.__dict__["_state"] = state

    def __repr__(self):
        return f"<inert {type(self).__name__}>"


def _placeholder(full_name: str):
    mod, _, name = full_name.rpartition(".")
    cls = type(name, (_Inert,), {"__module__": mod})
    cls.__qualname__ = name
    return cls


def _allowed(full_name: str) -> bool:
    return any(full_name.startswith(p) for p in ALLOWED_PREFIXES)


def load_checkpoint_objects(path) -> dict:
    """torch.load(path, weights_only=True) with inert placeholders for the reference's classes."""
    path = str(path)
    names = torch.serialization.get_unsafe_globals_in_checkpoint(path)
    bad = sorted(n for n in names if not _allowed(n))
    if bad:
        raise RuntimeError(f"checkpoint {path} names globals outside the allowed families: {bad[:8]}")
    stubs = [(_placeholder(n), n) for n in names]
    with torch.serialization.safe_globals(stubs):
        return torch.load(path, map_location="cpu", weights_only=True)


def _module_state(obj, prefix: str, out: dict):
    d = getattr(obj, "__dict__", {})
    skip = d.get("_non_persistent_buffers_set") or set()
    if isinstance(skip, _Inert):  # a set pickled by REDUCE(builtins.set, [names])
        skip = set(skip.__dict__.get("_args", ((),))[0])
    for k, v in (d.get("_parameters") or {}).items():
        if isinstance(v, torch.Tensor):
            out[prefix + k] = v
    for k, v in (d.get("_buffers") or {}).items():
        if isinstance(v, torch.Tensor) and k not in skip:
            out[prefix + k] = v
    for k, m in (d.get("_modules") or {}).items():
        if m is not None:
            _module_state(m, f"{prefix}{k}.", out)


def read_reference_checkpoint(path) -> dict:
    """-> {"state_dict": fp32 tensors with the reference's key names, "yaml": dict | None,
    "names": dict | None, "train_args": dict | None}.  Also accepts plain state_dict files."""
    p = Path(path)
    if not p.exists():
        raise FileNotFoundError(path)
    ckpt = load_checkpoint_objects(p)
    if isinstance(ckpt, dict) and all(isinstance(v, torch.Tensor) for v in ckpt.values()):
        return {"state_dict": {k: v.float() for k, v in ckpt.items()}, "yaml": None, "names": None,
                "train_args": None}
    if not isinstance(ckpt, dict):
        raise ValueError(f"{path}: expected a checkpoint dict, got {type(ckpt).__name__}")
    model = ckpt.get("ema") or ckpt.get("model")
    if model is None:
        raise ValueError(f"{path}: checkpoint holds neither 'ema' nor 'model'")
    if isinstance(model, dict):  # exported state_dict under "model"
        sd = model
        yaml_d = ckpt.get("yaml")
        names = ckpt.get("names")
    else:
        sd = {}
        _module_state(model, "", sd)
        md = model.__dict__
        yaml_d = md.get("yaml")
        names = md.get("names")
    if not sd:
        raise ValueError(f"{path}: no parameters found in the checkpoint model")
    args = ckpt.get("train_args")
    return {"state_dict": {k: v.float() if v.is_floating_point() else v for k, v in sd.items()},
            "yaml": dict(yaml_d) if isinstance(yaml_d, dict) else None,
            "names": dict(names) if isinstance(names, dict) else None,
            "train_args": dict(args) if isinstance(args, dict) else None}
