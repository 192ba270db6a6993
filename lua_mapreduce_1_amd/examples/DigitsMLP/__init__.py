"""Iterative MapReduce training of the digits MLP — the reference's APRIL-ANN
example (/root/reference/mapreduce/examples/APRIL-ANN/{init,common,server,
worker}.lua).  One module provides every function (pass it as taskfn, mapfn,
partitionfn, reducefn and finalfn), in two execution forms:

* server/worker — ``init_args = [connection_string, data, max_epochs?]``
  (``data``: a digits.png-shaped file or ``"synthetic"``): the reference's
  shape, described below;
* SPMD on the device data plane — ``init_args = {"data": ..., "max_epochs":
  ...}`` through ``execute_spmd.py`` / ``lua_mapreduce_1_amd.spmd``: the map
  jobs' gradients are emitted as fp32 tensors per weight name into the
  tensor plane (``device_reduce = "tensor_sum"``, parallel/tensor_plane.py),
  reduced by ONE RCCL reduce-scatter by weight-name partition and one
  all-gather, and ``device_finalfn`` steps the replicated model on every rank
  — no gradient bytes through the host (``HISTORY`` keeps the epochs).

* ``init``: opens the persistent table ``conf`` and, if there is no model (or the
  previous run finished), creates one and checkpoints it to the coordinator's
  blob store (common.lua:57-77; ``serialize_to_gridfs`` :24-29).  Checkpoints
  are ``.npz`` data (loaded with ``allow_pickle=False``), never executable.
* ``taskfn``: 4 map jobs per iteration (init.lua:65-70).
* ``mapfn``: reload the model when ``conf.version`` changed, gradient of one
  random bunch of 128 patterns — the fused MFMA kernel on a GPU worker — and emit
  one record per weight name plus ``TR_LOSS`` (common.lua:85-104).
* ``partitionfn``: byte sum of the key mod 10 (common.lua:106-109).
* ``reducefn``: sum gradients and bunch counts, accumulate the loss
  (common.lua:112-137).
* ``finalfn``: 1/sqrt(N) smoothing, SGD step, validation, checkpoint, and
  ``"loop"`` until the stopping rule says stop (common.lua:144-202).
"""
from __future__ import annotations

import io
import math

import numpy as np
import torch

from lua_mapreduce_1_amd import persistent_table
from lua_mapreduce_1_amd.models import mlp_dpsgd as T
from lua_mapreduce_1_amd.ops import mlp as M
from lua_mapreduce_1_amd.runtime.cnn import cnn as cnn_cls
from lua_mapreduce_1_amd.utils import digits

NUM_REDUCERS = 10
DB = "exp_digits"
TR_LOSS_KEY = "TR_LOSS"
STATE_BLOB = "digits_mlp.state"

CONN = None
DATA = "synthetic"
MAX_EPOCHS = None
conf = None
_data_cache: dict = {}
_trainer = None
_trainer_version = None
# SPMD form: replicated per rank (trainer, epoch, stopping rule, history)
SPMD = False
HISTORY: list = []
_spmd: dict = {}
device_reduce = "tensor_sum"   # the SPMD tensor plane; a server/worker run takes the host mapfn
spmd_replicated_taskfn = True


def _device():
    return "cuda" if torch.cuda.is_available() else "cpu"


def _blobs():
    return cnn_cls(CONN, DB).gridfs()


def _save_state(tr: T.DigitsTrainer) -> None:
    buf = io.BytesIO()
    np.savez(buf, w=tr.w.cpu().numpy(), v=tr.v.cpu().numpy())
    g = _blobs()
    g.remove_file(STATE_BLOB)
    g.store_data(buf.getvalue(), STATE_BLOB)


def _load_trainer() -> T.DigitsTrainer:
    """The model at ``conf.version`` (cached per process)."""
    global _trainer, _trainer_version
    if _trainer is not None and _trainer_version == conf.version:
        return _trainer
    raw = _blobs().get(STATE_BLOB)
    if raw is None:
        raise RuntimeError("model checkpoint missing from the blob store")
    with np.load(io.BytesIO(raw), allow_pickle=False) as z:
        w, v = torch.from_numpy(z["w"]), torch.from_numpy(z["v"])
    hyper = {"max_epochs": MAX_EPOCHS} if MAX_EPOCHS else None
    if _trainer is None:
        _trainer = T.DigitsTrainer(_device(), _dataset(DATA), hyper, params=w)
    else:
        _trainer.w.copy_(w.to(_trainer.device))
    _trainer.v.copy_(v.to(_trainer.device))
    _trainer_version = conf.version
    return _trainer


def _dataset(value):
    if value not in _data_cache:
        _data_cache[value] = digits.load(None if value == "synthetic" else value)
    return _data_cache[value]


def init(arg):
    global CONN, DATA, MAX_EPOCHS, conf, SPMD, HISTORY
    if isinstance(arg, dict):
        # SPMD form: every rank holds the (identical) model; nothing shared
        SPMD = True
        DATA = arg.get("data", DATA) or "synthetic"
        MAX_EPOCHS = int(arg["max_epochs"]) if arg.get("max_epochs") else None
        HISTORY = []
        _spmd.clear()
        return
    SPMD = False
    arg = list(arg or [])
    if arg:
        CONN = arg[0]
    if len(arg) > 1 and arg[1]:
        DATA = arg[1]
    if len(arg) > 2 and arg[2]:
        MAX_EPOCHS = int(arg[2])
    conf = persistent_table("conf", CONN, DB)
    if conf.version is None or conf.finished:
        if conf.finished:
            conf.drop()
            g = _blobs()
            for f in g.list():
                g.remove_file(f["filename"])
        tr = T.DigitsTrainer("cpu", _dataset(DATA), None)
        _save_state(tr)
        st = tr.stop
        conf.set({"finished": False, "version": 0, "epoch": 0, "best_epoch": 0, "best_val": None,
                  "history": [], "min_epochs": st.min_epochs,
                  "max_epochs": MAX_EPOCHS or st.max_epochs})
        conf.update()


def taskfn(emit):
    if not SPMD:
        conf.update()
    for j in range(1, T.HYPER["jobs_per_iteration"] + 1):
        emit(j, DATA)


# -- SPMD form: the tensor plane ------------------------------------------------------
def device_tensor_layout() -> dict:
    """Keys and sizes of the tensor plane: one fp32 gradient per weight name
    and [loss, correct, count] under TR_LOSS (common.lua:95-103)."""
    lay = {name: getattr(M.LAYOUT, name).stop - getattr(M.LAYOUT, name).start for name in M.WEIGHT_NAMES}
    lay[TR_LOSS_KEY] = 3
    return lay


def _spmd_trainer(device) -> T.DigitsTrainer:
    tr = _spmd.get("trainer")
    if tr is None:
        hyper = {"max_epochs": MAX_EPOCHS} if MAX_EPOCHS else None
        tr = _spmd["trainer"] = T.DigitsTrainer(device, _dataset(DATA), hyper)
        _spmd["epoch"] = 0
    return tr


def device_mapfn(key, value, emit):
    """The gradient of map job ``key``'s bunch (the fused MFMA kernel on a
    GPU) into the tensor plane, per weight name (common.lua:85-104)."""
    tr = _spmd_trainer(emit.device)
    tr.compute_gradients(tr.bunch_indices(_spmd["epoch"] + 1, [key]))
    for name in M.WEIGHT_NAMES:
        emit.tensor(name, tr.grads[getattr(M.LAYOUT, name)])
    emit.tensor(TR_LOSS_KEY, tr.buf[-3:])


def device_finalfn(res, engine):
    """Every rank: the summed gradients (res.tensors, device) -> 1/sqrt(N)
    smoothing + SGD step, validation, stopping rule (common.lua:144-202);
    the same on every rank, so the replicated model stays identical."""
    tr = _spmd_trainer(engine.device)
    grads = tr.grads  # (free after the map: the flat gradient the SGD kernel reads)
    for name in M.WEIGHT_NAMES:
        grads[getattr(M.LAYOUT, name)].copy_(res.tensors[name])
    loss, correct, count = res.tensors[TR_LOSS_KEY].tolist()  # 3 floats: the stopping rule's input
    tr.apply(grads, count)
    va_loss, va_acc = tr.validate()
    tr_loss = loss / max(count, 1.0)
    go = tr.stop.update(tr_loss, va_loss)
    _spmd["epoch"] += 1
    HISTORY.append({"epoch": _spmd["epoch"], "tr_loss": tr_loss, "va_loss": va_loss, "va_acc": va_acc,
                    "tr_acc": correct / max(count, 1.0)})
    if engine.rank == 0 and engine.verbose:
        print(tr.stop.state_string(), flush=True)
    return "loop" if go else True


def mapfn(key, value, emit):
    conf.update()
    tr = _load_trainer()
    idx = tr.bunch_indices(conf.epoch + 1, [key])
    tr.compute_gradients(idx)
    buf = tr.buf.cpu().numpy()
    n = M.LAYOUT.size
    flat = buf[:n]
    count = int(buf[-1])
    for name in M.WEIGHT_NAMES:
        sl = getattr(M.LAYOUT, name)
        emit(name, (flat[sl].tobytes(), count))
    emit(TR_LOSS_KEY, (float(buf[-3]), float(buf[-2]), count))


def partitionfn(key):
    return sum(key.encode()) % NUM_REDUCERS


def reducefn(key, values, emit):
    if key == TR_LOSS_KEY:
        emit((sum(v[0] for v in values), sum(v[1] for v in values), sum(v[2] for v in values)))
        return
    g = np.frombuffer(values[0][0], dtype=np.float32).copy()
    count = values[0][1]
    for v in values[1:]:
        g += np.frombuffer(v[0], dtype=np.float32)
        count += v[1]
    emit((g.tobytes(), count))


def finalfn(pairs):
    conf.update()
    tr = _load_trainer()
    grads = torch.zeros(M.LAYOUT.size, dtype=torch.float32)
    tr_loss = None
    count = 0
    for key, values in pairs:
        v = values[0]
        if key == TR_LOSS_KEY:
            tr_loss = v[0] / max(v[2], 1)
            continue
        sl = getattr(M.LAYOUT, key)
        grads[sl] = torch.from_numpy(np.frombuffer(v[0], dtype=np.float32).copy())
        count = max(count, v[1])
    if tr_loss is None:
        raise RuntimeError("finalfn: no training loss received")
    tr.apply(grads.to(tr.device), count)
    va_loss, va_acc = tr.validate()
    stop = T.StopRule(conf.min_epochs, conf.max_epochs, epoch=conf.epoch, best_epoch=conf.best_epoch,
                      best_val=math.inf if conf.best_val is None else conf.best_val)
    go = stop.update(tr_loss, va_loss)
    _save_state(tr)
    conf.set({"version": conf.version + 1, "epoch": stop.epoch, "best_epoch": stop.best_epoch,
              "best_val": stop.best_val, "history": list(conf.history) + [[stop.epoch, tr_loss, va_loss, va_acc]]})
    print(stop.state_string(), flush=True)
    if go:
        conf.update()
        return "loop"
    conf.set({"finished": True})
    conf.update()
    return True
