"""Checkpoint / resume (the reference has none — ``lightning_learner.py:85`` disables it).

The checkpoint format *is* the reference wire format: ``P2PFLModel.encode_parameters()`` =
``pickle({"params": [ndarray…], "additional_info": {…}})`` (``p2pfl_model.py:81-85``), so a
checkpoint can be sent to a reference node and a reference weights message can be loaded as a
checkpoint. Client-side callback state (SCAFFOLD ``c_i``) rides in ``additional_info`` under
``"_callback_state"``. A JSON sidecar holds experiment name, completed rounds, epochs, contributors,
the Settings snapshot and RNG states.

Layout::

    <dir>/<exp_name>/<node-addr>/round_<r>.bin    (wire bytes)
    <dir>/<exp_name>/<node-addr>/round_<r>.json   (sidecar)
    <dir>/<exp_name>/<node-addr>/latest.json      (pointer to the newest round)

Loading uses the safe unpickler (``p2pfl_model.safe_loads``): nothing in the file is executed.
Resume: ``restore_node(node, path)`` then ``node.set_start_learning(rounds, epochs,
start_round=meta["round"])``.
"""

from __future__ import annotations

import base64
import json
import os
import random
import re
from typing import Any, Dict, Optional, Tuple

import numpy as np

from myfyp_amd.learning.frameworks.p2pfl_model import safe_loads
from myfyp_amd.settings import Settings

_CB_KEY = "_callback_state"


def _slug(addr: str) -> str:
    return re.sub(r"[^A-Za-z0-9_.-]", "_", addr)


def node_dir(directory: str, exp_name: str, addr: str) -> str:
    return os.path.join(directory, _slug(exp_name), _slug(addr))


def _rng_state() -> Dict[str, Any]:
    import torch

    st: Dict[str, Any] = {
        "python": repr(random.getstate()),
        "numpy": json.loads(json.dumps(np.random.get_state(legacy=False), default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o))),
        "torch": base64.b64encode(torch.get_rng_state().numpy().tobytes()).decode(),
    }
    return st


def _restore_rng(st: Dict[str, Any]) -> None:
    import ast

    import torch

    if "python" in st:
        random.setstate(ast.literal_eval(st["python"]))
    if "numpy" in st:
        s = st["numpy"]
        s["state"]["key"] = np.asarray(s["state"]["key"], dtype=np.uint32) if "key" in s.get("state", {}) else s.get("state")
        np.random.set_state(s)
    if "torch" in st:
        torch.set_rng_state(torch.from_numpy(np.frombuffer(base64.b64decode(st["torch"]), dtype=np.uint8).copy()))


def save_checkpoint(learner, directory: str, exp_name: str, addr: str, round: int, total_rounds: Optional[int] = None, epochs: Optional[int] = None) -> str:
    """Write ``round_<round>.{bin,json}`` for one node; returns the ``.bin`` path."""
    model = learner.get_model()
    info = dict(model.get_info() or {})
    cb_state = {cb.get_name(): cb.state_dict() for cb in getattr(learner, "callbacks", [])}
    cb_state = {k: v for k, v in cb_state.items() if v}
    if cb_state:
        info[_CB_KEY] = cb_state
    blob = model.encode_parameters() if not cb_state else _encode_with_info(model, info)
    d = node_dir(directory, exp_name, addr)
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"round_{round}.bin")
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(blob)
    os.replace(tmp, path)
    meta = {
        "format": "p2pfl-pickle-v1",
        "exp_name": exp_name,
        "addr": addr,
        "round": round,
        "total_rounds": total_rounds,
        "epochs": epochs if epochs is not None else getattr(learner, "epochs", None),
        "num_samples": int(getattr(model, "num_samples", 0) or 0),
        "contributors": list(getattr(model, "contributors", []) or []),
        "framework": model.get_framework(),
        "settings": Settings.snapshot(),
        "rng": _rng_state(),
    }
    with open(os.path.join(d, f"round_{round}.json"), "w") as f:
        json.dump(meta, f, indent=1)
    with open(os.path.join(d, "latest.json"), "w") as f:
        json.dump({"round": round, "path": os.path.basename(path)}, f)
    return path


def _encode_with_info(model, info: Dict[str, Any]) -> bytes:
    import pickle

    from myfyp_amd.learning.frameworks.p2pfl_model import _to_host

    return pickle.dumps({"params": model.get_parameters(), "additional_info": _to_host(info)})


def latest_checkpoint(directory: str, exp_name: str, addr: str) -> Optional[str]:
    d = node_dir(directory, exp_name, addr)
    p = os.path.join(d, "latest.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return os.path.join(d, json.load(f)["path"])


def load_checkpoint(path: str) -> Tuple[list, Dict[str, Any], Dict[str, Any]]:
    """Return ``(params, additional_info, meta)``; meta is ``{}`` for a bare wire blob."""
    with open(path, "rb") as f:
        obj = safe_loads(f.read())
    if not isinstance(obj, dict) or "params" not in obj:
        raise ValueError(f"{path}: not a p2pfl parameter blob")
    meta: Dict[str, Any] = {}
    side = path[: -len(".bin")] + ".json" if path.endswith(".bin") else None
    if side and os.path.exists(side):
        with open(side) as f:
            meta = json.load(f)
    return obj["params"], dict(obj.get("additional_info") or {}), meta


def restore_learner(learner, path: str, restore_rng: bool = False) -> Dict[str, Any]:
    """Load a checkpoint into a learner (model params + callback state); returns the sidecar."""
    params, info, meta = load_checkpoint(path)
    cb_state = info.pop(_CB_KEY, {})
    model = learner.get_model()
    model.set_parameters(params)
    for k, v in info.items():
        model.add_info(k, v)
    if meta.get("contributors"):
        model.set_contribution(meta["contributors"], int(meta.get("num_samples") or 0))
    learner.set_model(model)
    for cb in getattr(learner, "callbacks", []):
        if cb.get_name() in cb_state:
            cb.load_state_dict(cb_state[cb.get_name()])
    if restore_rng and "rng" in meta:
        _restore_rng(meta["rng"])
    return meta


def restore_node(node, path: Optional[str] = None, directory: Optional[str] = None, exp_name: Optional[str] = None, restore_rng: bool = False) -> Dict[str, Any]:
    """Restore a node from ``path`` or from its newest checkpoint under ``directory``."""
    if path is None:
        if directory is None:
            raise ValueError("path or directory required")
        path = latest_checkpoint(directory, exp_name or node.exp_name, node.addr)
        if path is None:
            raise FileNotFoundError(f"no checkpoint for {node.addr} under {directory}")
    return restore_learner(node.learner, path, restore_rng=restore_rng)


def maybe_checkpoint(state, learner) -> Optional[str]:
    """Called by ``RoundFinishedStage`` after ``increase_round``: honours ``Settings.CHECKPOINT_DIR``
    and ``Settings.CHECKPOINT_EVERY`` (the final round is always saved)."""
    directory = Settings.CHECKPOINT_DIR
    if not directory or state.round is None:
        return None
    every = max(1, int(Settings.CHECKPOINT_EVERY))
    if state.round % every and state.round != state.total_rounds:
        return None
    return save_checkpoint(learner, directory, state.exp_name or "experiment", state.addr, state.round, state.total_rounds, getattr(learner, "epochs", None))
