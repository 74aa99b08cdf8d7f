"""Grouped fused MLP engine: co-located peers trained by ONE sequence of HIP launches.

This replaces the reference's per-node Lightning ``Trainer`` (``lightning_learner.py:78-108``) and
the Ray actor pool (``simulation/actor_pool.py``) for ReLU MLPs on MI355X:

* every peer of the same architecture/batch size on a device gets a *slot* in one stacked
  ``[capacity, S]`` fp32 parameter buffer (+ Adam moments, bf16 shadow, W2ᵀ shadow); the peer's
  ``nn.Module`` parameters are views into its row, so ``state_dict``/wire format are unchanged;
* ``fit`` calls from the peers' learning threads are *ganged*: the first arrival opens a batch,
  which closes when every expected co-located peer arrived (or ``Settings.GANG_WINDOW`` passed);
  one thread then runs the whole batch — each local epoch is ONE ``hipGraphLaunch`` of the C++
  engine (``csrc/runtime/engine.hip``) whose kernels cover all peers via ``grid.z``;
* ``evaluate`` is ganged the same way (one forward sweep over every peer's test split).

Numerics (``Settings.MLP_PRECISION``): "fp32" (default, the reference's precision — Lightning's
default fp32 Trainer, ``lightning_learner.py:82-89``) runs the fp32 persistent epoch
(``csrc/kernels/mlp_persistent_f32.hip``: exact fp32 products, fp32 accumulation, fp32 weights and
optimizer state) and the fp32 evaluation; "bf16" uses bf16 MFMA operands with fp32 accumulation,
master weights and optimizer state. Both follow the ``torch.optim.Adam``/``SGD`` update rules with
fresh optimizer state per ``fit`` (Lightning semantics).
"""

from __future__ import annotations

import ctypes
import os
import random
import threading
import time
from typing import Dict, List, Optional, Set, Tuple

import numpy as np
import torch

from myfyp_amd.utils.seed import seed_generation

from myfyp_amd.ops import _native
from myfyp_amd.parallel.pending import Pending, Resolver
from myfyp_amd.settings import Settings


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def mlp_dims(module: torch.nn.Module) -> Optional[Tuple[int, int, int, int]]:
    """(D0, D1, D2, D3) of a 3-Linear ReLU MLP (the reference architecture family) else None."""
    from myfyp_amd.models.mlp import MLP

    if not isinstance(module, MLP) or module.activation != "relu" or len(module.hidden_sizes) != 2:
        return None
    lins = module.linear_layers()
    if any(lin.bias is None for lin in lins):
        return None
    return (lins[0].in_features, lins[0].out_features, lins[1].out_features, lins[2].out_features)


class _CallTimer:
    """Diagnostics (env ``MYFYP_TIME_CALLS=<path>``): host time between marks of the round's engine
    calls, per label, summed over the run and written as JSON at exit."""

    def __init__(self) -> None:
        import os

        self.path = os.environ.get("MYFYP_TIME_CALLS")
        self.on = bool(self.path)
        self.tot: Dict[str, list] = {}
        self._t = threading.local()
        if self.on:
            import atexit

            atexit.register(self.dump)

    def mark(self, label: Optional[str]) -> None:
        if not self.on:
            return
        now = time.perf_counter()
        last = getattr(self._t, "t", None)
        if label is not None and last is not None:
            ent = self.tot.setdefault(label, [0, 0.0])
            ent[0] += 1
            ent[1] += now - last
        self._t.t = now

    def dump(self) -> None:
        import json

        with open(self.path, "w") as f:
            json.dump({k: {"calls": n, "us_mean": round(1e6 * t / max(1, n), 2)} for k, (n, t) in sorted(self.tot.items())}, f, indent=1)


_CALL_T = _CallTimer()


class _DeviceCtx:
    """``torch.cuda.device`` without its per-call overhead (the round driver enters it once per
    group and round): exchange the thread's current device on entry, restore it on exit."""

    __slots__ = ("idx", "prev")

    def __init__(self, idx: int) -> None:
        self.idx = idx
        self.prev = -1

    def __enter__(self):
        self.prev = torch.cuda._exchange_device(self.idx) if self.idx >= 0 else -1
        return self

    def __exit__(self, *exc) -> None:
        if self.idx >= 0:
            torch.cuda._maybe_exchange_device(self.prev)


class _Gang:
    """Collects requests from co-located peers' threads and runs them as one batch."""

    def __init__(self, run_batch, live_fn=None) -> None:
        self._run_batch = run_batch
        self._live_fn = live_fn  # slots still attached (a stopped peer is never waited for)
        self._cv = threading.Condition()
        self._pending: Dict[int, object] = {}
        self._results: Dict[int, object] = {}
        self._errors: Dict[int, BaseException] = {}
        self._running = False
        self._t_first = 0.0
        self.expected: Optional[Set[int]] = None

    def submit(self, slot: int, req: object, default_expected: Set[int]) -> object:
        window = Settings.GANG_WINDOW
        with self._cv:
            if not self._pending:
                self._t_first = time.time()
            self._pending[slot] = req
            self._cv.notify_all()
            while slot not in self._results and slot not in self._errors:
                expected = self.expected if self.expected is not None else default_expected
                if self._live_fn is not None:
                    expected = expected & self._live_fn()
                complete = expected.issubset(self._pending.keys())
                waited = time.time() - self._t_first
                if not self._running and self._pending and (complete or waited >= window):
                    batch, self._pending = self._pending, {}
                    self._running = True
                    self._cv.release()
                    try:
                        results = self._run_batch(batch)
                        errors: Dict[int, BaseException] = {}
                    except BaseException as e:  # propagate to every member of the batch
                        results, errors = {}, {s: e for s in batch}
                    finally:
                        self._cv.acquire()
                        self._running = False
                    self._results.update(results)
                    self._errors.update(errors)
                    if self._pending:
                        self._t_first = time.time()
                    self._cv.notify_all()
                else:
                    self._cv.wait(timeout=max(0.0005, window - waited) if not self._running else 0.05)
            if slot in self._errors:
                raise self._errors.pop(slot)
            return self._results.pop(slot)

    def poke(self) -> None:
        with self._cv:
            self._cv.notify_all()


class MLPGroup:
    """All peers of one (device, dims, batch size) — one native engine, one stacked buffer."""

    _groups: Dict[tuple, "MLPGroup"] = {}
    _lock = threading.Lock()

    @classmethod
    def get(cls, device: torch.device, dims: Tuple[int, int, int, int], batch_size: int, precision: Optional[str] = None, tag=None) -> "MLPGroup":
        """``tag``: the peers' device-mesh rank (a virtual mesh puts several ranks on one GPU)."""
        precision = precision or Settings.MLP_PRECISION
        key = (str(device), dims, batch_size, precision, tag)
        with cls._lock:
            g = cls._groups.get(key)
            if g is None:
                with torch.cuda.device(device):
                    g = cls(device, dims, batch_size, precision=precision)
                g.mesh_rank = tag
                cls._groups[key] = g
            return g

    @classmethod
    def reset_all(cls) -> None:
        with cls._lock:
            for g in cls._groups.values():
                g.close()
            cls._groups.clear()

    def __init__(self, device: torch.device, dims: Tuple[int, int, int, int], batch_size: int, capacity: int = 8, precision: str = "fp32") -> None:
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"MLP precision must be 'fp32' or 'bf16', got {precision!r}")
        self.precision = precision
        self.device = device
        self.mesh_rank = None
        self.dims = dims
        self.B = batch_size
        D0, D1, D2, D3 = dims
        self.numel = D1 * D0 + D1 + D2 * D1 + D2 + D3 * D2 + D3
        self.S = (self.numel + 63) // 64 * 64
        self.lock = threading.RLock()
        self.handles: Dict[int, "MLPEngineHandle"] = {}
        self.capacity = 0
        self._engine = None
        self._engine_cap = 0
        self._data_version = 0
        self._bound_version = -1
        self.extras: Dict[str, torch.Tensor] = {}
        self.perm_fn = None  # test hook: callable(epoch) -> int32 [capacity, nmax] permutation
        self.eager = False  # debug/profiling A-B: launch steps without the hipGraph
        self.force_f32_ks: Optional[int] = None  # test hook: fp32 owner K split (1, 2, 4, 8)
        # test / A-B hook: fp32 gang layout (1 owners + heads, 2 owners only; None = default)
        self.force_f32_variant: Optional[int] = None
        # weight-stationary persistent epoch kernel (csrc/kernels/mlp_persistent.hip): None = auto
        # (used whenever the shape/optimizer is eligible), False = always the 3-launch step path
        self.persistent: Optional[bool] = None
        self._fedavg_buf: Optional[torch.Tensor] = None
        self._alloc(capacity)
        self.fit_gang = _Gang(self._run_fit_batch, lambda: set(self.handles))
        self.eval_gang = _Gang(self._run_eval_batch, lambda: set(self.handles))
        # asynchronous results: pinned ring slots on the engine, resolved in order by ONE thread per
        # process (shared by every group: a device mesh has one group per GPU, and a resolver thread
        # each would contend for the GIL with the round driver)
        self.resolver = Resolver.shared()
        self._cfg_key: Optional[tuple] = None  # last engine configuration pushed to the native side
        self._seed_ahead: Optional[int] = None  # shuffle key of the next epoch (its gather is already enqueued)
        self._seed_gen = -1  # utils.seed.seed_generation() the key above was drawn under
        self._opt_key: Optional[tuple] = None
        self._steps_pe: Optional[np.ndarray] = None
        self._active_cache: Dict[tuple, np.ndarray] = {}
        self._ring = 0
        self._next_slot = 0
        self._slot_free: List[threading.Event] = []

    # ------------------------------------------------------------------ buffers / slots
    def _alloc(self, capacity: int) -> None:
        old = (getattr(self, "params", None), getattr(self, "m", None), getattr(self, "v", None))
        dev = self.device
        D1, D2 = self.dims[1], self.dims[2]
        params = torch.zeros(capacity, self.S, dtype=torch.float32, device=dev)
        if old[0] is not None:
            params[: self.capacity].copy_(old[0])
        self.params = params
        self.m = torch.zeros_like(params)
        self.v = torch.zeros_like(params)
        self.shadow = torch.zeros(capacity, self.S, dtype=torch.bfloat16, device=dev)
        self.w2t = torch.zeros(capacity, D1 * D2, dtype=torch.bfloat16, device=dev)
        self.capacity = capacity
        for slot, h in self.handles.items():
            h.flat.retarget(self.params[slot, : self.numel])
        self._close_engine()

    def _close_engine(self) -> None:
        if self._engine is not None:
            _native.load(required=True).mlp_engine_destroy(self._engine)
            self._engine = None
        self._cfg_key = self._opt_key = None

    def close(self) -> None:
        self._close_engine()

    def attach(self, handle: "MLPEngineHandle") -> int:
        with self.lock:
            slot = next((i for i in range(self.capacity) if i not in self.handles), None)
            if slot is None:
                self._alloc(self.capacity * 2)
                slot = next(i for i in range(self.capacity) if i not in self.handles)
            self.handles[slot] = handle
            self._data_version += 1
            return slot

    def detach(self, slot: int) -> None:
        with self.lock:
            self.handles.pop(slot, None)
            self._data_version += 1
        self.fit_gang.poke()
        self.eval_gang.poke()

    def invalidate_data(self) -> None:
        with self.lock:
            self._data_version += 1
            self._seed_ahead = None  # the key drawn ahead belonged to the old data

    # ------------------------------------------------------------------ native engine
    def _ensure_engine(self) -> None:
        lib = _native.load(required=True)
        if self._engine is None or self._engine_cap != self.capacity:
            self._close_engine()
            D0, D1, D2, D3 = self.dims
            eng = lib.mlp_engine_create(self.capacity, D0, D1, D2, D3, self.B)
            if not eng:
                raise RuntimeError(f"mlp_engine_create failed: {lib.myfyp_last_error().decode()}")
            self._engine = eng
            self._engine_cap = self.capacity
            self._bound_version = -1
            _native.check(
                lib.mlp_engine_bind_params(eng, _p(self.params), _p(self.shadow), _p(self.w2t), _p(self.m), _p(self.v), self.S), "bind_params"
            )
        # fp32 owner K split: 1 (24-workgroup gangs). Each gang then runs on ONE XCD and keeps its
        # hand-offs in that XCD's L2 (csrc/kernels/persist_common.h gang_same_xcd), which beats
        # K split 2's halved owner work on 40-workgroup gangs that must span two XCDs: 601-607 vs
        # 570-578 rounds/s at 4 / 2 / 1 peers per GPU (profiles/r5_ksab). With the hand-offs forced
        # write-through (MYFYP_F32_PLAIN_PUB=0) the old choice: 2 when every peer sits in the first
        # 4 slots (one launch covers them all)
        #
        # Round 6: with at most 4 peers on the device, a peer's gang spans 8 / peers XCDs instead (the
        # cross-XCD K split, csrc/kernels/mlp_persistent_f32.hip "XR"): the K parts of a column
        # group reduce inside one XCD, and only the H1 and dH2 hand-offs cross XCDs. That puts the
        # XCDs an 8-peer GPU gives to the other peers on this peer's critical path (N = 2 / 4 / 8
        # GPUs hold 4 / 2 / 1 peers each). MYFYP_F32_XSPLIT=0 keeps K split 1.
        if self.force_f32_ks:
            ks = self.force_f32_ks
        elif os.environ.get("MYFYP_F32_XSPLIT", "1") != "0" and self.B == 64 and self.handles:
            # measured (profiles/r6_xr): 1 peer K split 8 628.8 vs 612.2 rounds/s at K split 1, 2 peers
            # K split 4 657.9 vs 622.7; 4 peers K split 2 612.8 vs 620.3 (loses: stays at 1)
            # peer slots on this PHYSICAL device: a virtual mesh puts several groups on one GPU,
            # whose launches then share its XCDs (one XCD per peer: K split 1)
            used = self._device_peer_slots()
            ks = 8 if used <= 1 else 4 if used <= 2 else 1
        else:
            ks = 1
        # a forced K split > 1 is a layout-1 configuration
        var = self.force_f32_variant or (1 if (self.force_f32_ks or 1) > 1 else 0)
        # weight collectives on the comm stream may hold CUs while an epoch runs: size the
        # co-resident gangs without them
        from myfyp_amd.parallel.federation import Federation, rccl_reserved_cus

        fed = Federation._instance
        reserve = rccl_reserved_cus() if fed is not None and not fed.solo else 0
        key = (self._engine, self.precision, ks, var, reserve, self.persistent)
        if key != self._cfg_key:  # the setters run only when something changed (host cost per round)
            _native.check(lib.mlp_engine_set_precision(self._engine, 1 if self.precision == "fp32" else 0), "set_precision")
            _native.check(lib.mlp_engine_set_f32_ks(self._engine, ks), "set_f32_ks")
            _native.check(lib.mlp_engine_set_f32_variant(self._engine, var), "set_f32_variant")
            _native.check(lib.mlp_engine_set_reserved_cus(self._engine, reserve), "set_reserved_cus")
            if self.persistent is not None:  # None: engine default (auto; env MYFYP_MLP_PERSISTENT=0 disables)
                _native.check(lib.mlp_engine_set_persistent(self._engine, -1 if self.persistent else 0), "set_persistent")
            self._cfg_key = key
        if self._bound_version != self._data_version:
            self._bind_data()
            self._bound_version = self._data_version
            self._steps_pe = None

    def _device_peer_slots(self) -> int:
        """Peer slots every MLP group on this group's physical device covers (its own launch's, plus
        those of the other mesh ranks a virtual mesh placed on the same GPU)."""
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        used = max(self.handles) + 1 if self.handles else 0
        with MLPGroup._lock:
            others = [g for g in MLPGroup._groups.values() if g is not self and g.device.type == "cuda"
                      and (g.device.index if g.device.index is not None else idx) == idx]
        for g in others:
            if g.handles:
                used += max(g.handles) + 1
        return max(1, used)

    def fedavg_buffer(self) -> torch.Tensor:
        """Device scratch of numel + 1 floats for the stacked FedAvg (weighted sum | Σw)."""
        if self._fedavg_buf is None or self._fedavg_buf.numel() != self.numel + 1:
            self._fedavg_buf = torch.empty(self.numel + 1, dtype=torch.float32, device=self.device)
        return self._fedavg_buf

    def uses_persistent(self) -> bool:
        """True if the next local epoch runs as the weight-stationary persistent kernel."""
        with self.lock, self.on_device():
            self._ensure_engine()
            return bool(_native.load(required=True).mlp_engine_uses_persistent(self._engine))

    def _bind_data(self) -> None:
        """(Re)build the per-peer data pointer tables (uploads each peer's split once)."""
        lib = _native.load(required=True)
        cap, dev = self.capacity, self.device
        xs, ys, ns, xts, yts, nts = [0] * cap, [0] * cap, [0] * cap, [0] * cap, [0] * cap, [0] * cap
        if self._engine is not None and getattr(self, "_keep", None):
            # a gather enqueued ahead on the engine's prep stream may still read the tensors bound
            # so far (the torch allocator does not track that stream): drain it before dropping them
            _native.check(lib.mlp_engine_drain_prep(self._engine), "drain_prep")
        self._seed_ahead = None
        self._keep = []
        for slot, h in self.handles.items():
            (x, y), (xt, yt) = h.device_split(True), h.device_split(False)
            xs[slot], ys[slot], ns[slot] = x.data_ptr(), y.data_ptr(), x.shape[0]
            xts[slot], yts[slot], nts[slot] = xt.data_ptr(), yt.data_ptr(), xt.shape[0]
            self._keep += [x, y, xt, yt]
        self.n_train = ns
        self.n_test = nts
        # builds with direct-X fp32 epochs (opt-in, -DP32_XDIRECT=1) read every batch row from an
        # exact bf16 copy of the peer's uint8 images (made once per data binding): [n_p][D0] per slot
        # (built whatever the precision: a later switch to fp32 must not find a missing table)
        x16s = [0] * cap
        want_x16 = bool(lib.mlp_engine_x_direct_build())
        for slot, h in (self.handles.items() if want_x16 else ()):
            x = h.device_split(True)[0]
            if x.shape[0] > 0:
                x16 = x.to(torch.bfloat16)
                x16s[slot] = x16.data_ptr()
                self._keep.append(x16)
        self._tables = {
            "Xp": torch.tensor(xs, dtype=torch.int64, device=dev),
            "Yp": torch.tensor(ys, dtype=torch.int64, device=dev),
            "n": torch.tensor(ns, dtype=torch.int32, device=dev),
            "Xtp": torch.tensor(xts, dtype=torch.int64, device=dev),
            "Ytp": torch.tensor(yts, dtype=torch.int64, device=dev),
            "nt": torch.tensor(nts, dtype=torch.int32, device=dev),
            "Xp16": torch.tensor(x16s, dtype=torch.int64, device=dev),
        }
        self.nmax = max(1, max(ns) if ns else 1)
        self.max_steps = (self.nmax + self.B - 1) // self.B
        self.perm = torch.zeros(cap, self.nmax, dtype=torch.int32, device=dev)
        t = self._tables
        _native.check(lib.mlp_engine_set_train_data(self._engine, _p(t["Xp"]), _p(t["Yp"]), _p(t["n"]), _p(self.perm), self.nmax, self.max_steps), "set_train_data")
        _native.check(lib.mlp_engine_set_test_data(self._engine, _p(t["Xtp"]), _p(t["Ytp"]), _p(t["nt"]), max(nts) if nts else 0), "set_test_data")
        _native.check(lib.mlp_engine_set_train_x16(self._engine, _p(t["Xp16"]) if want_x16 else None), "set_train_x16")
        n_host = np.asarray(ns, dtype=np.int32)
        nt_host = np.asarray(nts, dtype=np.int32)
        _native.check(lib.mlp_engine_set_counts(self._engine, n_host.ctypes.data, nt_host.ctypes.data), "set_counts")

    def _extra_buffer(self, name: str) -> torch.Tensor:
        buf = self.extras.get(name)
        if buf is None or buf.shape[0] != self.capacity:
            buf = torch.zeros(self.capacity, self.S, dtype=torch.float32, device=self.device)
            self.extras[name] = buf
        return buf

    def _set_optimizer(self, lib, spec: dict, mu: float, anchor, cg, cl) -> None:
        key = (self._engine, tuple(sorted(spec.items())), mu, _p(anchor), _p(cg), _p(cl), self.perm_fn is None)
        if key == self._opt_key:
            return
        self._opt_key = key
        _native.check(lib.mlp_engine_set_shuffle(self._engine, 0 if self.perm_fn is not None else 1), "set_shuffle")
        kind = 0 if spec.get("name", "adam") == "adam" else 1
        _native.check(
            lib.mlp_engine_set_optimizer(
                self._engine, kind, float(spec.get("lr", 1e-3)) * _native.debug_update_scale(), float(spec.get("beta1", 0.9)), float(spec.get("beta2", 0.999)),
                float(spec.get("eps", 1e-8)), float(spec.get("weight_decay", 0.0)), float(spec.get("momentum", 0.0)),
                int(bool(spec.get("nesterov", False))), mu,
            ),
            "set_optimizer",
        )
        _native.check(lib.mlp_engine_set_extras(self._engine, _p(anchor), _p(cg), _p(cl)), "set_extras")

    def on_device(self):
        """Make the group's GPU current for this thread (the native engine allocates and captures
        on the current device; a process may drive several devices: parallel/device_mesh.py)."""
        return _DeviceCtx(self.device.index if self.device.index is not None else -1)

    def _active(self, slots) -> np.ndarray:
        """int32 active mask over the capacity for ``slots`` (cached: the same sets recur every round)."""
        key = tuple(sorted(slots))
        a = self._active_cache.get(key)
        if a is None or a.shape[0] != self.capacity:
            a = np.zeros(self.capacity, dtype=np.int32)
            a[list(key)] = 1
            if len(self._active_cache) > 64:
                self._active_cache.clear()
            self._active_cache[key] = a
        return a

    def prewarm(self, spec: dict) -> None:
        """One-time engine setup before the first fit (node start): bind the data, capture and
        upload the epoch graph for ``spec`` (no FedProx/SCAFFOLD extras: those re-capture on their
        first fit), allocate the evaluation side and load the code object. Runs no training work;
        a later change (another peer attaching, other optimizer settings) re-captures as before."""
        lib = _native.load(required=True)
        with self.lock, self.on_device():
            _native.warm_device(torch.cuda.current_device())
            self._ensure_engine()
            self._set_optimizer(lib, spec, 0.0, None, None, None)
            _native.check(lib.mlp_engine_prepare(self._engine, torch.cuda.current_stream(self.device).cuda_stream), "prepare")

    # ------------------------------------------------------------------ batched fit
    def _run_fit_batch(self, batch: Dict[int, tuple]) -> Dict[int, tuple]:
        lib = _native.load(required=True)
        _CALL_T.mark(None)
        with self.lock, self.on_device():
            self._ensure_engine()
            stream = torch.cuda.current_stream(self.device).cuda_stream
            specs = list(batch.values())
            spec, epochs = specs[0][0], max(r[1] for r in specs)
            extras_any = [r[2] for r in specs if r[2]]
            mu = 0.0
            anchor = cg = cl = None
            if any("anchor" in e for e in extras_any):
                anchor = self._extra_buffer("anchor")
                mu = float(next(e["mu"] for e in extras_any if "anchor" in e))
            if any("c_global" in e for e in extras_any):
                cg, cl = self._extra_buffer("c_global"), self._extra_buffer("c_local")
            for slot, (_, _, extra) in batch.items():
                if anchor is not None:
                    anchor[slot, : self.numel].copy_(extra["anchor"] if "anchor" in extra else self.params[slot, : self.numel])
                if cg is not None:
                    if "c_global" in extra:
                        cg[slot, : self.numel].copy_(extra["c_global"])
                        cl[slot, : self.numel].copy_(extra["c_local"])
                    else:
                        cg[slot].zero_()
                        cl[slot].zero_()
            fast = _native.load_fast()
            # (also sets the shuffle mode: the epoch order is drawn on the device inside the gather
            # kernel — keyed Feistel permutation per peer, key from the seeded Python RNG — unless a
            # test pins explicit permutations)
            self._set_optimizer(fast, spec, mu, anchor, cg, cl)
            active = self._active(batch)
            _CALL_T.mark("fit_prep")
            # fresh optimizer state per fit (Lightning semantics); slots not training this round are
            # zeroed as well — they start fresh when they next train — so this is 2 memsets, not 2P
            _native.check(fast.mlp_engine_zero_state(self._engine, stream), "zero_state")
            _native.check(fast.mlp_engine_begin(self._engine, active.ctypes.data, stream), "begin")
            _CALL_T.mark("fit_zero_begin")
            if self._steps_pe is None:
                self._steps_pe = np.array([(n + self.B - 1) // self.B for n in self.n_train], dtype=np.int32)
            steps_pe = self._steps_pe
            # the result slot is taken first: the last epoch's graph publishes into it itself (its
            # last node), so stats_async is then a no-op — no separate launch behind the graph
            k = self._take_slot()
            _CALL_T.mark("fit_take_slot")
            try:
                for ep in range(epochs):
                    if self.perm_fn is not None:
                        self.perm.copy_(self.perm_fn(ep))
                        self._seed_ahead = None
                    else:
                        # keys are drawn one epoch ahead: the engine enqueues the next epoch's gather
                        # right after launching this one (same keys, same order as drawing each in
                        # turn within one RNG stream; a set_seed() in between drops the key ahead)
                        gen = seed_generation()
                        if gen != self._seed_gen:
                            self._seed_ahead, self._seed_gen = None, gen
                        seed = self._seed_ahead if self._seed_ahead is not None else random.getrandbits(64)
                        self._seed_ahead = random.getrandbits(64)
                        _native.check(fast.mlp_engine_set_epoch_seed(self._engine, seed), "set_epoch_seed")
                        _native.check(fast.mlp_engine_set_next_epoch_seed(self._engine, self._seed_ahead), "set_next_epoch_seed")
                    t0 = steps_pe if ep == 1 else (steps_pe * ep).astype(np.int32)
                    if self.eager:
                        _native.check(fast.mlp_engine_run_epoch_eager(self._engine, t0.ctypes.data, stream), "run_epoch")
                    else:
                        _CALL_T.mark("fit_seed")
                        _native.check(fast.mlp_engine_run_epoch_pub(self._engine, t0.ctypes.data, k if ep == epochs - 1 else -1, stream), "run_epoch")
                        _CALL_T.mark("fit_run_epoch")
                _native.check(fast.mlp_engine_stats_async(self._engine, k, stream), "stats_async")
                _CALL_T.mark("fit_stats_async")
            except BaseException:
                self._slot_free[k].set()  # nothing will fetch this slot: give it back to the ring
                raise
            raw = self.resolver.submit(lambda k=k: self._fetch(k, with_conf=False))
            _CALL_T.mark("fit_submit")
        out = {}
        for slot in batch:
            n = max(1, self.n_train[slot] * epochs)
            out[slot] = (int(steps_pe[slot] * epochs), raw.map(lambda r, s=slot, n=n: (float(r[0][s]) / n, float(r[1][s]) / n)))
        return out

    # ------------------------------------------------------------------ result ring
    def _take_slot(self) -> int:
        lib = _native.load(required=True)
        if not self._slot_free:
            self._ring = int(lib.mlp_engine_ring_size())
            self._slot_free = [threading.Event() for _ in range(self._ring)]
            for e in self._slot_free:
                e.set()
        k = self._next_slot % self._ring
        self._next_slot += 1
        if not self._slot_free[k].wait(timeout=Settings.AGGREGATION_TIMEOUT):
            raise RuntimeError("device result ring stalled")
        self._slot_free[k].clear()
        return k

    def _fetch(self, k: int, with_conf: bool):
        lib = _native.load(required=True)
        loss = np.zeros(self.capacity, dtype=np.float32)
        correct = np.zeros(self.capacity, dtype=np.int32)
        conf = np.zeros((self.capacity, 16, 16), dtype=np.int32) if with_conf else None
        before = self.recoveries()
        try:
            _native.check(lib.mlp_engine_fetch(self._engine, k, loss.ctypes.data, correct.ctypes.data, conf.ctypes.data if with_conf else None), "fetch")
        finally:
            self._slot_free[k].set()
        if self.recoveries() != before:
            from myfyp_amd.management.logger import logger

            logger.warning("mlp-engine", "persistent epoch: a gang gave up (workgroup not resident) and was re-run by the retry launch")
        return loss, correct, conf

    def epoch_launch_kind(self) -> str:
        """How a local epoch reaches the GPU: the persistent epoch kernel is launched directly
        (engine.hip ``direct_epoch_launch``; ``MYFYP_EPOCH_GRAPH=1`` replays its captured graph
        instead); the step path replays a captured hipGraph."""
        if self.uses_persistent() and os.environ.get("MYFYP_EPOCH_GRAPH", "0") in ("", "0"):
            return "persistent-direct"
        return ("persistent-" if self.uses_persistent() else "steps-") + "hipgraph"

    def f32_variant(self) -> int:
        """Gang layout the fp32 persistent epoch uses (1 owners + heads, 2 owners only)."""
        with self.lock, self.on_device():
            self._ensure_engine()
            return int(_native.load(required=True).mlp_engine_f32_variant(self._engine))

    def f32_ks(self) -> int:
        """Owner K split the fp32 persistent epoch uses (1, or 2 / 4 / 8: the cross-XCD K split)."""
        with self.lock, self.on_device():
            self._ensure_engine()
            return int(_native.load(required=True).mlp_engine_f32_ks(self._engine))

    def graph_launch_stats(self) -> dict:
        """Host time inside hipGraphLaunch (launches, mean / max us) and the number of alternating
        epoch-graph executables."""
        if not self._engine:
            return {}
        out = np.zeros(3, dtype=np.uint64)
        n = int(_native.load(required=True).mlp_engine_graph_launch_stats(self._engine, out.ctypes.data))
        k = max(1, int(out[0]))
        return {"execs": n, "launches": int(out[0]), "mean_us": round(float(out[1]) / k / 1e3, 2), "max_us": round(float(out[2]) / 1e3, 2)}

    def recoveries(self) -> int:
        """Give-ups of the persistent fp32 epoch that the in-stream retry launch recovered."""
        return int(_native.load(required=True).mlp_engine_recoveries(self._engine)) if self._engine else 0

    def debug_giveup(self, slot: Optional[int], at_end: bool = False) -> None:
        """Test hook: the peer in ``slot`` gives up on the first attempt of every fp32 epoch, at
        launch or (``at_end``) at the gang commit after its last step."""
        with self.lock, self.on_device():
            self._ensure_engine()
            _native.check(_native.load(required=True).mlp_engine_debug_giveup(self._engine, -1 if slot is None else int(slot), int(at_end)), "debug_giveup")

    def _run_eval_batch(self, batch: Dict[int, tuple]) -> Dict[int, tuple]:
        lib = _native.load(required=True)
        _CALL_T.mark(None)
        with self.lock, self.on_device():
            self._ensure_engine()
            stream = torch.cuda.current_stream(self.device).cuda_stream
            active = self._active(batch)
            k = self._take_slot()
            # GIL kept (PyDLL): the call only enqueues, except that on the overlapped path it may poll
            # (host side, bounded by GPU progress alone) for the evaluation two rounds back to release
            # its snapshot side. Releasing the GIL here handed it to other threads for up to the
            # switch interval per group and round (device mesh: 8 groups per round)
            _CALL_T.mark("eval_prep")
            _native.check(_native.load_fast().mlp_engine_eval_async(self._engine, active.ctypes.data, k, stream), "eval_async")
            _CALL_T.mark("eval_async")
            raw = self.resolver.submit(lambda k=k: self._fetch(k, with_conf=True))
            _CALL_T.mark("eval_submit")
        D3 = self.dims[3]
        return {slot: raw.map(lambda r, s=slot: (float(r[0][s]) / max(1, self.n_test[s]), r[2][s, :D3, :D3].copy())) for slot in batch}

    def expect(self, fit_slots: Optional[Set[int]] = None, eval_slots: Optional[Set[int]] = None) -> None:
        """Tell the gangs exactly which slots will call (collective workflow knows it)."""
        self.fit_gang.expected = fit_slots
        self.eval_gang.expected = eval_slots

    def default_expected(self) -> Set[int]:
        return set(self.handles)


def feistel_perm(x: int, n: int, key: int) -> int:
    """Host mirror of the gather kernel's epoch permutation (``feistel_perm`` in mlp_fused.hip):
    4-round balanced Feistel network on the smallest even bit width covering n, cycle-walked."""
    if n <= 1:
        return 0
    bits = max(2, (n - 1).bit_length())
    bits += bits & 1
    half = bits // 2
    mask = (1 << half) - 1
    k0, k1 = key & 0xFFFFFFFF, (key >> 32) & 0xFFFFFFFF

    def mix32(v: int) -> int:
        v &= 0xFFFFFFFF
        v ^= v >> 16
        v = (v * 0x7FEB352D) & 0xFFFFFFFF
        v ^= v >> 15
        v = (v * 0x846CA68B) & 0xFFFFFFFF
        v ^= v >> 16
        return v

    y = x
    while True:
        lo, hi = y & mask, y >> half
        left, right = hi, lo
        for r in range(4):
            f = mix32(right ^ (k1 if r & 1 else k0) ^ ((0x9E3779B9 * (r + 1)) & 0xFFFFFFFF)) & mask
            left, right = right, left ^ f
        y = (left << half) | right
        if y < n:
            return y


class _RetargetableFlat:
    """Parameter views of one module into a row of the group buffer."""

    def __init__(self, module: torch.nn.Module, storage: torch.Tensor) -> None:
        self.module = module
        self.params = [p for p in module.parameters()]
        self.retarget(storage, copy_in=True)

    def retarget(self, storage: torch.Tensor, copy_in: bool = False) -> None:
        off = 0
        with torch.no_grad():
            for p in self.params:
                view = storage[off : off + p.numel()].view_as(p)
                if copy_in:
                    view.copy_(p.data.to(view.dtype))
                p.data = view
                off += p.numel()
        self.flat = storage


class MLPEngineHandle:
    """A learner's slot in an :class:`MLPGroup`."""

    @staticmethod
    def supports(module: torch.nn.Module, batch_size: Optional[int] = None) -> bool:
        dims = mlp_dims(module)
        if dims is None:
            return False
        lib = _native.load()
        if lib is None:
            # GPU + fused path requested but no library: fail loudly (no silent eager fallback)
            raise RuntimeError(f"MI355X fused engine requested but native library unavailable: {_native.error()}")
        if Settings.MLP_PRECISION == "fp32":
            # the fp32 engine has no bf16 fallback: shapes it cannot run stay on fp32 autograd
            return bool(lib.mlp_f32_ok(*dims, int(batch_size or Settings.BATCH_SIZE)))
        return bool(lib.mlp_shape_ok(*dims))

    @classmethod
    def attach(cls, module: torch.nn.Module, device: torch.device, addr: str, learner=None, batch_size: Optional[int] = None, tag=None) -> "MLPEngineHandle":
        return cls(module, device, addr, int(batch_size or Settings.BATCH_SIZE), learner, tag)

    def __init__(self, module: torch.nn.Module, device: torch.device, addr: str, batch_size: int, learner=None, tag=None) -> None:
        self.addr = addr
        self.module = module
        self.group = MLPGroup.get(device, mlp_dims(module), batch_size, tag=tag)
        self.learner = learner
        self._data_id = id(learner.data) if learner is not None else None
        with self.group.lock:
            self.slot = self.group.attach(self)
            self.flat = _RetargetableFlat(module, self.group.params[self.slot, : self.group.numel])

    def close(self) -> None:
        self.group.detach(self.slot)

    def flat_params(self) -> torch.Tensor:
        return self.flat.flat

    def device_split(self, train: bool) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.learner is None or self.learner.data is None:
            D0 = self.group.dims[0]
            return torch.zeros(0, D0, dtype=torch.uint8, device=self.group.device), torch.zeros(0, dtype=torch.int32, device=self.group.device)
        x, y = self.learner.device_data(train, label_dtype=torch.int32)
        x = x.reshape(x.shape[0], -1)
        if x.dtype != torch.uint8:
            raise TypeError("fused MLP engine expects uint8 images")
        if not x.is_contiguous():
            x = x.contiguous()
        return x, y

    def fit(self, learner, spec: dict, extra: dict) -> Tuple[int, float]:
        if self.learner is not learner or getattr(self, "_data_id", None) != id(learner.data):
            self.learner = learner
            self._data_id = id(learner.data)
            self.group.invalidate_data()
        steps, stats = self.group.fit_gang.submit(self.slot, (spec, learner.epochs, extra), self.group.default_expected())
        learner.global_step += steps
        return steps, stats.map(lambda v: v[0])  # mean train loss, resolved asynchronously

    def evaluate(self, learner) -> "Pending":
        """Enqueue the grouped evaluation; the returned Pending resolves to (mean NLL, confusion)."""
        if self.learner is not learner or getattr(self, "_data_id", None) != id(learner.data):
            self.learner = learner
            self._data_id = id(learner.data)
            self.group.invalidate_data()
        return self.group.eval_gang.submit(self.slot, (), self.group.default_expected())
