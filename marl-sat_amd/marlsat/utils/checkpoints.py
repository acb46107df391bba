"""Checkpoints in the reference's on-disk format (flax.training.checkpoints, msgpack).

The reference saves ``runner_state.train_state`` every update with
``checkpoints.save_checkpoint(ckpt_dir, target, step=0, prefix="latest_model_",
overwrite=True)`` (runner:373-381) and restores it the same way (runner:204-231,
:387-397); BC pre-training writes ``bc_model_*`` with target ``{"params": ...}``
(model_init.py, runner:233-261).  flax writes ``flax.serialization.to_bytes(target)``
to ``<ckpt_dir>/<prefix><step>``: msgpack of the target's state dict, where every
array is a msgpack ExtType(1, packb((shape, dtype_name, raw C-order bytes))), numpy
scalars ExtType(3, ...), tuples become {"0": .., "1": ..} and NamedTuples dicts of
their fields.  A TrainState's state dict is
    {"step": int, "params": <param tree>,
     "opt_state": {"0": {"count": i32, "mu": <tree>, "nu": <tree>},   # optax.scale_by_adam
                   "1": {"count": i32} (LR schedule) | {} (constant LR)}}.
flax is not installed here, so this layout is restated from flax's serialization
rules (flax 0.8-0.10, requirements.txt) -- parity unpinned: no reference checkpoint
ships with the reference repo.  Loading uses msgpack with an ext hook only (no code
execution).
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import msgpack
import numpy as np

EXT_NDARRAY, EXT_COMPLEX, EXT_NPSCALAR = 1, 2, 3


# ---------------------------------------------------------------- codec ----
def _pack_ext(x):
    if isinstance(x, np.ndarray):
        return msgpack.ExtType(EXT_NDARRAY, msgpack.packb((x.shape, x.dtype.name, x.tobytes("C")), use_bin_type=True))
    if isinstance(x, np.generic):
        return msgpack.ExtType(EXT_NPSCALAR, msgpack.packb((x.dtype.name, x.tobytes()), use_bin_type=True))
    if isinstance(x, complex):
        return msgpack.ExtType(EXT_COMPLEX, msgpack.packb((x.real, x.imag)))
    raise TypeError(f"cannot serialise {type(x)}")


def _unpack_ext(code, data):
    if code == EXT_NDARRAY:
        shape, name, buf = msgpack.unpackb(data, raw=False)
        return np.frombuffer(buf, dtype=np.dtype(name)).reshape(shape).copy()
    if code == EXT_NPSCALAR:
        name, buf = msgpack.unpackb(data, raw=False)
        return np.frombuffer(buf, dtype=np.dtype(name))[0]
    if code == EXT_COMPLEX:
        re, im = msgpack.unpackb(data, raw=False)
        return complex(re, im)
    return msgpack.ExtType(code, data)


def to_bytes(state_dict) -> bytes:
    return msgpack.packb(state_dict, default=_pack_ext, strict_types=True)


def from_bytes(data: bytes):
    return msgpack.unpackb(data, ext_hook=_unpack_ext, raw=False)


# ------------------------------------------------------------ trees ----
def nest(flat: Dict[str, np.ndarray]) -> Dict:
    """{"encoder/update_c/ir/kernel": a} -> {"encoder": {"update_c": {"ir": {"kernel": a}}}}."""
    out: Dict = {}
    for k, v in flat.items():
        d = out
        parts = k.split("/")
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = np.asarray(v)
    return out


def flatten(tree: Dict, prefix: str = "") -> Dict[str, np.ndarray]:
    out = {}
    for k, v in tree.items():
        key = f"{prefix}/{k}" if prefix else k
        if isinstance(v, dict):
            out.update(flatten(v, key))
        else:
            out[key] = v
    return out


# ------------------------------------------------------- train state ----
def train_state_dict(net, lr_schedule: bool = True) -> Dict:
    """The device network's parameters + Adam state as a flax TrainState state dict."""
    import torch  # noqa: F401  (net tensors live on the device)

    from ..learners import params as P

    def tree_of(buf):
        flat = P.to_flax(buf.detach().cpu().numpy(), net.H, net.L, net.A, net.M, net.mode, net.E)
        return nest({k: v.astype(np.float32) for k, v in flat.items()})

    count = np.asarray(net.adam_count, dtype=np.int32)
    return {
        "step": np.asarray(net.adam_count, dtype=np.int32),
        "params": tree_of(net.params),
        "opt_state": {"0": {"count": count, "mu": tree_of(net.adam_m), "nu": tree_of(net.adam_v)},
                      "1": {"count": count} if lr_schedule else {}},
    }


def load_train_state(net, state: Dict, reset_optimizer: bool = False) -> None:
    """Restore params (and, unless reset_optimizer, the Adam moments / count) into the device net."""
    import torch

    from ..learners import params as P

    def buf_of(tree):
        return torch.from_numpy(P.from_flax(flatten(tree), net.H, net.L, net.A, net.M, net.mode, net.E))

    net.params.copy_(buf_of(state["params"]))
    if reset_optimizer:
        net.adam_m.zero_()
        net.adam_v.zero_()
        net.adam_count = 0
        return
    adam = state["opt_state"]["0"]
    net.adam_m.copy_(buf_of(adam["mu"]))
    net.adam_v.copy_(buf_of(adam["nu"]))
    net.adam_count = int(np.asarray(adam["count"]))


def save_checkpoint(ckpt_dir: str, target: Dict, step: int = 0, prefix: str = "latest_model_",
                    overwrite: bool = True) -> str:
    """flax.training.checkpoints.save_checkpoint analogue: writes <ckpt_dir>/<prefix><step> atomically."""
    os.makedirs(ckpt_dir, exist_ok=True)
    path = os.path.join(ckpt_dir, f"{prefix}{step}")
    if os.path.exists(path) and not overwrite:
        raise FileExistsError(path)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(to_bytes(target))
    os.replace(tmp, path)
    return path


def restore_checkpoint(ckpt_dir: str, prefix: str = "latest_model_", step: Optional[int] = 0) -> Optional[Dict]:
    """Returns the state dict of <ckpt_dir>/<prefix><step> (latest step when step is None), or None."""
    if not os.path.isdir(ckpt_dir):
        return None
    if step is None:
        steps = [int(f[len(prefix):]) for f in os.listdir(ckpt_dir)
                 if f.startswith(prefix) and f[len(prefix):].isdigit()]
        if not steps:
            return None
        step = max(steps)
    path = os.path.join(ckpt_dir, f"{prefix}{step}")
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        return from_bytes(f.read())


def inject_bc(net, bc_state: Dict) -> None:
    """runner:233-261: copy encoder + actor / agent-embedding params of a BC checkpoint
    ({"params": ...}); the critic keeps its init; the optimizer is reset."""
    cur = train_state_dict(net)["params"]
    bc = bc_state["params"]
    cur["encoder"] = bc["encoder"]
    for k in bc:
        if "actor" in k or "agent_id_embedding" in k:
            cur[k] = bc[k]
    load_train_state(net, {"params": cur}, reset_optimizer=True)
