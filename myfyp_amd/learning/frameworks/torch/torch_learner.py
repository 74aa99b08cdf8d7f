"""PyTorch-ROCm learner (parity: ``p2pfl/learning/frameworks/pytorch/lightning_learner.py:43-152``).

What the reference does through Lightning (new ``Trainer`` per ``fit``, Adam re-created per fit,
batch size 1, ``train_loss`` per step, ``test_loss``/``test_metric`` on evaluate) is done here
without Lightning, designed for the GPU:

* the node's partition is uploaded to HBM once (``uint8`` images + labels) and mini-batches are
  gathered on device — no DataLoader, no per-sample host work;
* trainable parameters live in one flat fp32 buffer (:class:`FlatParams`) and the optimizer is
  one fused HIP launch (``ops.adam_step`` / ``ops.sgd_step``) with the FedProx / SCAFFOLD
  corrections fused in;
* ReLU MLPs on a GPU bypass autograd entirely: the grouped fused engine
  (:mod:`myfyp_amd.parallel.mlp_engine`) runs whole epochs as replayed HIP graphs of
  hand-written MFMA kernels, batching all co-located peers into each launch;
* metrics are reduced on device and synchronised once per epoch (the reference's per-step
  ``self.log`` forces a host sync per step).

Evaluation returns ``test_loss``, ``test_metric`` (accuracy, reference keys) plus the FYP metrics
``test_accuracy``, ``test_f1``, ``test_precision``, ``test_recall`` (macro, ``mlp_pytorch.txt:117-144``).
"""

from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from myfyp_amd import ops
from myfyp_amd.learning.frameworks import Framework
from myfyp_amd.learning.frameworks.learner import Learner
from myfyp_amd.learning.frameworks.p2pfl_model import P2PFLModel
from myfyp_amd.learning.frameworks.torch.torch_model import TorchModel
from myfyp_amd.management.logger import logger
from myfyp_amd.parallel.flat_params import FlatParams
from myfyp_amd.parallel.pending import Pending, resolve
from myfyp_amd.settings import Settings, resolve_device
from myfyp_amd.management.tracing import traced


def classification_metrics(confusion: np.ndarray) -> Dict[str, float]:
    """Accuracy + macro precision/recall/F1 from a ``[C, C]`` confusion matrix (rows = truth)."""
    cm = confusion.astype(np.float64)
    tp = np.diag(cm)
    pred = cm.sum(0)
    true = cm.sum(1)
    total = cm.sum()
    with np.errstate(divide="ignore", invalid="ignore"):
        prec = np.where(pred > 0, tp / pred, 0.0)
        rec = np.where(true > 0, tp / true, 0.0)
        f1 = np.where(prec + rec > 0, 2 * prec * rec / (prec + rec), 0.0)
    present = true > 0
    acc = float(tp.sum() / total) if total else 0.0
    return {
        "accuracy": acc,
        "precision": float(prec[present].mean()) if present.any() else 0.0,
        "recall": float(rec[present].mean()) if present.any() else 0.0,
        "f1": float(f1[present].mean()) if present.any() else 0.0,
    }


class TorchLearner(Learner):
    """Trains a ``TorchModel`` on the node's device."""

    def __init__(self, model: TorchModel, data=None, self_addr: str = "unknown-node", aggregator=None, batch_size: Optional[int] = None, device: Optional[str] = None,
                 mesh_rank: Optional[int] = None) -> None:
        super().__init__(model, data, self_addr, aggregator)
        self.device = torch.device(device or resolve_device())
        # rank of this peer's device in the process's device mesh (parallel/device_mesh.py); None
        # outside a mesh. Peers of one mesh rank share one stacked engine group.
        self.mesh_rank = mesh_rank
        self.batch_size = int(batch_size or Settings.BATCH_SIZE)
        self._interrupt = threading.Event()
        self._data_cache: Dict[tuple, Tuple[torch.Tensor, torch.Tensor]] = {}
        self._data_key: Optional[int] = None
        self.global_step = 0
        self._engine = None  # fused grouped engine handle (set by _maybe_attach_engine)
        self._flat: Optional[FlatParams] = None
        self._attach_module(model)

    def close(self) -> None:
        """Release the grouped-engine slot (called by ``Node.stop``); the learner keeps working on
        a private copy of its parameters."""
        if self._engine is not None:
            eng, self._engine = self._engine, None
            module = self.model.get_model()
            with torch.no_grad():
                for p in module.parameters():
                    p.data = p.data.clone()
                for name, b in list(module.named_buffers()):
                    if b.is_floating_point():
                        b.data = b.data.clone()
            eng.close()
            self._flat = FlatParams(module)

    # ------------------------------------------------------------------ model plumbing
    def _attach_module(self, model: TorchModel) -> None:
        module = model.get_model()
        if module is None:
            raise ValueError("TorchLearner needs a TorchModel wrapping an nn.Module")
        module.to(self.device)
        self._engine = self._maybe_attach_engine(module)
        if self._engine is None:
            self._flat = FlatParams(module)

    def _maybe_attach_engine(self, module: torch.nn.Module):
        if self.device.type != "cuda" or not Settings.USE_FUSED_KERNELS:
            return None
        from myfyp_amd.parallel.cnn_engine import CNNEngineHandle
        from myfyp_amd.parallel.mlp_engine import MLPEngineHandle

        if MLPEngineHandle.supports(module, self.batch_size):
            with torch.cuda.device(self.device):
                return MLPEngineHandle.attach(module, self.device, self._self_addr, learner=self, batch_size=self.batch_size, tag=self.mesh_rank)
        for handle in (CNNEngineHandle,):
            if handle.supports(module):
                with torch.cuda.device(self.device):
                    return handle.attach(module, self.device, self._self_addr, learner=self, batch_size=self.batch_size, tag=self.mesh_rank)
        return None

    def flat_params(self) -> torch.Tensor:
        if self._engine is not None:
            return self._engine.flat_params()
        assert self._flat is not None
        return self._flat.flat

    def split_flat(self, flat: torch.Tensor) -> List[torch.Tensor]:
        """Views of a flat trainable vector aligned with ``state_dict`` order (zeros for buffers)."""
        module = self.model.get_model()
        trainable = {id(p): p for p in module.parameters() if p.requires_grad}
        out: List[torch.Tensor] = []
        off = 0
        names = dict(module.named_parameters())
        for name, t in module.state_dict(keep_vars=True).items():
            p = names.get(name)
            if p is not None and id(p) in trainable:
                out.append(flat[off : off + p.numel()].view_as(p))
                off += p.numel()
            else:
                out.append(torch.zeros_like(t, dtype=torch.float32))
        return out

    def set_addr(self, addr: str) -> None:
        super().set_addr(addr)
        if self._engine is not None:
            self._engine.addr = addr

    def set_model(self, model) -> None:
        if isinstance(model, P2PFLModel) and model is not self.model:
            # copy values into the live (device-resident) module; keep metadata
            self.model.set_parameters(model.get_parameters())
            self.model.additional_info.update(model.additional_info)
            self.model.contributors = list(model.contributors)
            self.model.num_samples = model.num_samples
            self.update_callbacks_with_model_info()
            return
        super().set_model(model)

    def set_data(self, data) -> None:
        super().set_data(data)
        self._data_cache.clear()
        if self._engine is not None:
            self._engine.group.invalidate_data()

    # ------------------------------------------------------------------ data
    def device_data(self, train: bool = True, label_dtype: torch.dtype = torch.int64) -> Tuple[torch.Tensor, torch.Tensor]:
        """(images, labels) of the split on the learner's device, cached per split and label dtype.
        Labels are converted on the host: the fused engines' int32 tables then cost no torch kernel
        at node start (a torch kernel's first launch in a process loads its code object: tens of
        ms on a fresh box, measured in ``profiles/r5_start``)."""
        key = id(self.data)
        if self._data_key != key:
            self._data_cache.clear()
            self._data_key = key
        ck = (train, label_dtype)
        if ck not in self._data_cache:
            xd = next((v[0] for k, v in self._data_cache.items() if k[0] == train), None)
            if xd is None:
                xd = torch.from_numpy(np.ascontiguousarray(self.data.column("image", train))).to(self.device)
            ny = {torch.int64: np.int64, torch.int32: np.int32}[label_dtype]
            y = torch.from_numpy(np.ascontiguousarray(self.data.column("label", train)).astype(ny))
            self._data_cache[ck] = (xd, y.to(self.device))
        return self._data_cache[ck]

    def num_train_samples(self) -> int:
        return self.data.get_num_samples(train=True)

    # ------------------------------------------------------------------ train
    def prewarm(self) -> None:
        """One-time fused-engine setup before learning starts (graph capture and upload, code-object
        load; no training work). Called by ``Node.start`` when ``Settings.ENGINE_PREWARM`` is set."""
        eng = self._engine
        group = getattr(eng, "group", None) if eng is not None else None
        if group is not None and hasattr(group, "prewarm"):
            group.prewarm(self._optimizer_spec())

    def _optimizer_spec(self) -> dict:
        module = self.model.get_model()
        spec = getattr(module, "optimizer_spec", None)
        return spec() if callable(spec) else {"name": "adam", "lr": 1e-3}

    def _gather_corrections(self) -> dict:
        extra: dict = {}
        for cb in self.callbacks:
            if hasattr(cb, "grad_correction"):
                extra.update(cb.grad_correction())
        return extra

    @traced("fit")
    def fit(self) -> P2PFLModel:
        self._interrupt.clear()
        for cb in self.callbacks:
            if hasattr(cb, "on_train_start"):
                cb.on_train_start(self)
        spec = self._optimizer_spec()
        t0 = time.time()
        if self._engine is not None:
            steps, mean_loss = self._engine.fit(self, spec, self._gather_corrections())
        else:
            steps, mean_loss = self._fit_autograd(spec)
        logger.log_timing(self._self_addr, "fit", time.time() - t0)
        return self._fit_done(steps, mean_loss, spec)

    def fit_request(self) -> Tuple[dict, int, dict]:
        """(optimizer spec, epochs, corrections) of a fit that a fused-round leader runs for this
        peer (collective workflow: evaluate + fit + FedAvg of all co-located peers in one gang op);
        the peer's own bookkeeping then happens in :meth:`_fit_done`."""
        self._interrupt.clear()
        return self._optimizer_spec(), self.epochs, self._gather_corrections()

    def _fit_done(self, steps: int, mean_loss, spec: dict) -> P2PFLModel:
        if mean_loss is not None:
            snap, addr, gs = logger.experiment_snapshot(self._self_addr), self._self_addr, self.global_step
            if isinstance(mean_loss, Pending):  # fused engine: logged when the device result lands
                mean_loss.map_off_thread(lambda v: logger.log_metric_at(addr, snap, "train_loss", float(v), step=gs))
            else:
                logger.log_metric_at(addr, snap, "train_loss", float(mean_loss), step=gs)
        for cb in self.callbacks:
            if hasattr(cb, "on_train_end"):
                cb.on_train_end(self, steps, float(spec.get("lr", 1e-3)))
        self.model.set_contribution([self._self_addr], self.num_train_samples())
        self.add_callback_info_to_model()
        return self.model

    def _fit_autograd(self, spec: dict) -> Tuple[int, Optional[float]]:
        assert self._flat is not None
        module = self.model.get_model()
        module.train()
        x_all, y_all = self.device_data(train=True)
        n = x_all.shape[0]
        fp = self._flat
        opt = spec.get("name", "adam")
        m = torch.zeros_like(fp.flat)
        v = torch.zeros_like(fp.flat) if opt == "adam" else None
        extra = self._gather_corrections()
        loss_sum = torch.zeros((), device=self.device)
        steps = 0
        gen = torch.Generator(device="cpu")
        gen.manual_seed(int(Settings.SEED or 0) * 1000003 + self.global_step)
        for _ in range(self.epochs):
            perm = torch.randperm(n, generator=gen).to(self.device)
            for s in range(0, n, self.batch_size):
                if self._interrupt.is_set():
                    break
                idx = perm[s : s + self.batch_size]
                fp.zero_grad()
                loss = F.cross_entropy(module(x_all[idx]), y_all[idx])
                loss.backward()
                steps += 1
                self.global_step += 1
                if opt == "adam":
                    ops.adam_step(
                        fp.flat, fp.grad, m, v, steps, lr=spec.get("lr", 1e-3), weight_decay=spec.get("weight_decay", 0.0),
                        anchor=extra.get("anchor"), c_global=extra.get("c_global"), c_local=extra.get("c_local"), mu=extra.get("mu", 0.0),
                    )
                else:
                    ops.sgd_step(
                        fp.flat, fp.grad, m, lr=spec.get("lr", 0.01), momentum=spec.get("momentum", 0.0), weight_decay=spec.get("weight_decay", 0.0),
                        anchor=extra.get("anchor"), c_global=extra.get("c_global"), c_local=extra.get("c_local"), mu=extra.get("mu", 0.0),
                    )
                loss_sum += loss.detach()
        mean = float(loss_sum) / max(1, steps)
        return steps, mean

    def interrupt_fit(self) -> None:
        """Stop the running fit (reference ``lightning_learner.py:110-114``): the autograd loop
        checks the flag every batch; a fused CNN fit already on the device stops at its next step
        (``CNNEngineHandle.interrupt``). A fused MLP epoch (~1.5 ms on the device) runs to its end."""
        self._interrupt.set()
        eng = self._engine
        if eng is not None and hasattr(eng, "interrupt"):
            eng.interrupt()

    # ------------------------------------------------------------------ evaluate
    @torch.no_grad()
    def evaluate_raw(self) -> Tuple[float, np.ndarray]:
        """(mean test NLL, confusion matrix [C, C])."""
        if self._engine is not None:
            return resolve(self._engine.evaluate(self))
        module = self.model.get_model()
        module.eval()
        x_all, y_all = self.device_data(train=False)
        if x_all.shape[0] == 0:
            return 0.0, np.zeros((1, 1))
        loss_sum = torch.zeros((), device=self.device, dtype=torch.float64)
        conf = None
        chunk = 4096
        for s in range(0, x_all.shape[0], chunk):
            out = module(x_all[s : s + chunk])
            y = y_all[s : s + chunk]
            loss_sum += F.cross_entropy(out.float(), y, reduction="sum").double()
            c = out.shape[1]
            if conf is None:
                conf = torch.zeros(c * c, device=self.device, dtype=torch.int64)
            conf += torch.bincount(y * c + out.argmax(1), minlength=c * c)
        assert conf is not None
        c = int(round(conf.numel() ** 0.5))
        return float(loss_sum) / x_all.shape[0], conf.view(c, c).cpu().numpy()

    @staticmethod
    def _results(loss: float, conf: np.ndarray) -> Dict[str, float]:
        m = classification_metrics(conf)
        return {
            "test_loss": float(loss),
            "test_metric": m["accuracy"],
            "test_accuracy": m["accuracy"],
            "test_f1": m["f1"],
            "test_precision": m["precision"],
            "test_recall": m["recall"],
        }

    def evaluate_async(self) -> Pending:
        """Enqueue the evaluation and return at once; the metrics are logged against the round in
        which it was issued when the device result lands (the round's hot path never waits for the
        GPU). ``evaluate()`` is this plus a wait."""
        t0 = time.time()
        if self.data is None or self.data.get_num_samples(train=False) == 0:
            return Pending.completed({})
        snap = logger.experiment_snapshot(self._self_addr)
        raw = self._engine.evaluate(self) if self._engine is not None else self.evaluate_raw()
        out = self._evaluate_done(raw, snap)
        logger.log_timing(self._self_addr, "evaluate", time.time() - t0)
        return out

    def _evaluate_done(self, raw, snap) -> Pending:
        """Metrics of an issued evaluation (``raw`` = (loss, confusion) or its Pending), logged under
        the experiment snapshot taken when it was issued."""
        if not isinstance(raw, Pending):
            raw = Pending.completed(raw)
        addr = self._self_addr

        def done(lc) -> Dict[str, float]:
            results = self._results(*lc)
            for k, v in results.items():
                logger.log_metric_at(addr, snap, k, v)
            return results

        return raw.map_off_thread(done)

    @traced("evaluate")
    def evaluate(self) -> Dict[str, float]:
        return self.evaluate_async().result()

    def get_framework(self) -> str:
        return Framework.PYTORCH.value
