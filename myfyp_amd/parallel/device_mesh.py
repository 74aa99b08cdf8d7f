"""In-process device mesh: one process drives G devices; weights move over RCCL (xGMI).

SURVEY §2.10 #2 / §7.3 / §7.4.2: the reference keeps all peers of a simulation in one process and
moves models with direct calls (``p2pfl/communication/protocols/memory/server_singleton.py:22-43``,
``test/node_test.py:79-132``). Here the peers of one process are placed round-robin over G MI355X
devices; the co-located peers of each device form one stacked engine group, and the weights plane
between devices is a set of G RCCL communicators created together (``ncclCommInitAll``) and driven
from ONE host thread inside ``ncclGroupStart/End`` (``csrc/runtime/rccl_mesh.hip``).

Two implementations of one interface:

* :class:`RcclMesh` — the C++ wrapper (real devices, each listed once);
* :class:`HostMesh` — the same collectives as torch ops over the member tensors, stream-ordered on
  the current streams. It serves CPU hosts (tests of the multi-device logic with ``cpu`` members)
  and *virtual* meshes whose members share one physical GPU (a one-GPU rehearsal of the N-device
  path; RCCL refuses two ranks on one device).

Every method takes one tensor per mesh rank (rank i's tensor lives on ``devices[i]``) and enqueues
on each device's current stream: nothing here waits for the GPU.
"""

from __future__ import annotations

import ctypes
import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

_DTYPE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4, torch.float64: 5, torch.uint8: 6}
_OPS = {"sum": 0, "max": 1, "min": 2, "avg": 3}

_SIGS = {
    "rmesh_last_error": (ctypes.c_char_p, []),
    "rmesh_version": (ctypes.c_int, []),
    "rmesh_create": (ctypes.c_void_p, [ctypes.c_int, ctypes.c_void_p]),
    "rmesh_size": (ctypes.c_int, [ctypes.c_void_p]),
    "rmesh_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "rmesh_allreduce": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "rmesh_broadcast": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]),
    "rmesh_allgather": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]),
    "rmesh_p2p": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "rmesh_fedavg": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p]),
    "rmesh_fedavg_retry": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "rmesh_fedavg_bucketed": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]),
    "rmesh_delayed_land": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "rmesh_fedavg_bucketed_retry": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "rmesh_check": (ctypes.c_int, [ctypes.c_void_p]),
    "rmesh_abort": (ctypes.c_int, [ctypes.c_void_p]),
    "rmesh_shrink": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "rmesh_rebuild": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "rmesh_debug_inject": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "rmesh_destroy": (None, [ctypes.c_void_p]),
}


class MeshError(RuntimeError):
    """A mesh collective failed (or the mesh was aborted)."""


def _bucket_ranges(n: int, bucket: int) -> List[Tuple[int, int]]:
    """[b0, b1) over n floats, every b0 a multiple of 4 (the native ``bucket_step``)."""
    step = max(4, (int(bucket) // 4) * 4)
    return [(b0, min(n, b0 + step)) for b0 in range(0, n, step)] or [(0, 0)]


def _ptrs(vals: Sequence[int]) -> ctypes.Array:
    return (ctypes.c_void_p * len(vals))(*vals)


def _stream_ptr(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0


class Marker:
    """Completion marker of a mesh member's queued work: an event recorded on the member device's
    current stream, or on ``stream`` (``cpu`` members complete synchronously)."""

    def __init__(self, dev: torch.device, stream=None) -> None:
        self.ev = None
        if dev.type == "cuda":
            with torch.cuda.device(dev):
                self.ev = torch.cuda.Event()
                self.ev.record(stream if stream is not None else torch.cuda.current_stream(dev))

    def query(self) -> bool:
        return True if self.ev is None else bool(self.ev.query())


class _Stalled(Marker):
    """A member that never completes (HostMesh fault hook)."""

    def __init__(self) -> None:
        self.ev = None

    def query(self) -> bool:
        return False


class DeviceMesh:
    """Common interface (see the module docstring)."""

    kind = "abstract"

    def __init__(self, devices: Sequence[torch.device]) -> None:
        self.devices: List[torch.device] = [torch.device(d) for d in devices]
        self.lock = threading.RLock()
        self.calls = 0
        self.shrinks = 0

    @property
    def size(self) -> int:
        return len(self.devices)

    def _check_members(self, ts: Sequence[torch.Tensor], what: str) -> None:
        if len(ts) != self.size:
            raise ValueError(f"{what}: {len(ts)} tensors for a mesh of {self.size}")
        for t, d in zip(ts, self.devices):
            if t.device != d and not (d.index is None and t.device.type == d.type):
                raise ValueError(f"{what}: tensor on {t.device}, mesh rank on {d}")
            if not t.is_contiguous():
                raise ValueError(f"{what}: tensors must be contiguous")

    # ------------------------------------------------------------------ interface
    def all_reduce_(self, ts: Sequence[torch.Tensor], op: str = "sum") -> None:
        raise NotImplementedError

    def broadcast_(self, ts: Sequence[torch.Tensor], root: int) -> None:
        raise NotImplementedError

    def all_gather_(self, outs: Sequence[torch.Tensor], ins: Sequence[torch.Tensor]) -> None:
        raise NotImplementedError

    def p2p_(self, ops: Sequence[Tuple[str, int, int, torch.Tensor]]) -> None:
        """``ops``: (``"send"`` | ``"recv"``, rank, peer, tensor); all in one group."""
        raise NotImplementedError

    def fedavg_stacked(self, params: Sequence[torch.Tensor], bufs: Sequence[torch.Tensor], P: Sequence[int], n: int,
                       ld: Sequence[int], w: np.ndarray, mask: np.ndarray, outs: Optional[Sequence[torch.Tensor]] = None) -> None:
        """FedAvg over the stacked groups (one per rank); see ``rmesh_fedavg``. With ``outs`` the
        all-reduce is out of place and ``bufs`` keep each rank's local partial sum (the input of
        :meth:`fedavg_retry`)."""
        raise NotImplementedError

    def fedavg_retry(self, params, bufs, outs, P, n: int, ld, mask: np.ndarray) -> None:
        """Re-run a FedAvg's all-reduce from the retained partial sums ``bufs`` over the CURRENT
        members (after a shrink) into ``outs``, then apply to the masked rows."""
        raise NotImplementedError

    def fedavg_bucketed(self, params, keeps, outs, P, n: int, ld, w: np.ndarray, mask: np.ndarray, comm_streams, bucket: int, apply: bool = True) -> None:
        """Bucketed, overlapped FedAvg (``rmesh_fedavg_bucketed``): per member the partial sums
        [Σw, pad x3 | Σ w x] (n + 4 floats) into ``keeps`` and the per-bucket all-reduces into
        ``outs``, on ``comm_streams``; with ``apply`` the member's compute stream waits per bucket
        and applies it, without (delayed averaging) nothing waits: :meth:`delayed_land` lands it."""
        raise NotImplementedError

    def delayed_land(self, params, snaps, outs, P, n: int, ld, ld_snap: int, mask: np.ndarray, have_avg: bool) -> None:
        """Per member, on the compute stream: (after the last bucketed exchange, if ``have_avg``)
        masked rows x += avg / Σw - snap, then snap = x (``rmesh_delayed_land``)."""
        raise NotImplementedError

    def fedavg_bucketed_retry(self, params, keeps, outs, P, n: int, ld, mask: np.ndarray, apply: bool = True) -> None:
        """Re-run a bucketed FedAvg's exchange from the retained ``keeps`` over the CURRENT members
        (after a shrink), on the compute streams, then apply (if ``apply``)."""
        raise NotImplementedError

    def marker(self, rank: int, stream=None) -> Marker:
        """Completion marker of everything queued so far on member ``rank``'s current stream (or
        on ``stream``, e.g. its comm stream)."""
        return Marker(self.devices[rank], stream)

    def check(self) -> None:
        pass

    def abort(self) -> None:
        pass

    def shrink(self, keep: Sequence[int]) -> None:
        """Rebuild over the surviving ranks ``keep`` (indices into ``devices``), renumbered in order;
        after a failure (the communicators are aborted, never waited for)."""
        raise NotImplementedError

    def rebuild(self, keep: Sequence[int]) -> None:
        """Rebuild a HEALTHY mesh over ``keep`` (a device whose last peer left). The caller has
        drained every member device; the communicators are destroyed, not aborted."""
        self.shrink(keep)

    def inject_error(self, rank: int) -> None:
        """Fault hook: :meth:`check` reports an asynchronous error on ``rank`` until a rebuild."""
        raise NotImplementedError

    def close(self) -> None:
        pass


class HostMesh(DeviceMesh):
    """Torch-op implementation (CPU members, or virtual members on one GPU)."""

    kind = "host"

    def __init__(self, devices: Sequence[torch.device]) -> None:
        super().__init__(devices)
        self._stalled: set = set()  # fault hook: members (by device position) that never complete
        self._injected: Optional[int] = None
        self.aborted = False

    def stall(self, rank: int) -> None:
        """Fault hook: member ``rank`` stops completing work (its markers and probes never fire),
        like a device stuck in a kernel."""
        self._stalled.add(int(rank))

    def marker(self, rank: int, stream=None) -> Marker:
        if rank in self._stalled:
            return _Stalled()
        return super().marker(rank, stream)

    def inject_error(self, rank: int) -> None:
        self._injected = int(rank)

    def check(self) -> None:
        if self.aborted:
            raise MeshError("host mesh was aborted (rebuild it with shrink)")
        if self._injected is not None:
            raise MeshError(f"rank {self._injected}: injected asynchronous error")

    def abort(self) -> None:
        self.aborted = True

    def all_reduce_(self, ts, op: str = "sum") -> None:
        self._check_members(ts, "all_reduce")
        self._live()
        with self.lock:
            self.calls += 1
            acc = ts[0].detach().clone()
            for t in ts[1:]:
                x = t.to(acc.device)
                if op in ("sum", "avg"):
                    acc.add_(x)
                elif op == "max":
                    torch.maximum(acc, x, out=acc)
                elif op == "min":
                    torch.minimum(acc, x, out=acc)
                else:
                    raise ValueError(op)
            if op == "avg":
                acc.div_(len(ts))
            for t in ts:
                t.copy_(acc.to(t.device))

    def broadcast_(self, ts, root: int) -> None:
        self._check_members(ts, "broadcast")
        self._live()
        with self.lock:
            self.calls += 1
            src = ts[root]
            for i, t in enumerate(ts):
                if i != root:
                    t.copy_(src.to(t.device))

    def all_gather_(self, outs, ins) -> None:
        self._check_members(ins, "all_gather")
        self._live()
        with self.lock:
            self.calls += 1
            cat = torch.cat([x.reshape(-1).to(ins[0].device) for x in ins])
            for o in outs:
                o.view(-1).copy_(cat.to(o.device))

    def p2p_(self, ops) -> None:
        self._live()
        with self.lock:
            self.calls += 1
            sends = {}
            for kind, rank, peer, t in ops:
                if kind == "send":
                    sends.setdefault((rank, peer), []).append(t)
            for kind, rank, peer, t in ops:
                if kind == "recv":
                    q = sends.get((peer, rank))
                    if not q:
                        raise MeshError(f"p2p: receive on rank {rank} from {peer} has no matching send")
                    t.copy_(q.pop(0).to(t.device))

    def _live(self) -> None:
        if self.aborted:
            raise MeshError("host mesh was aborted (rebuild it with shrink)")

    def fedavg_stacked(self, params, bufs, P, n, ld, w, mask, outs=None) -> None:
        self._live()
        if all(t.is_cuda for t in params):
            return self._fedavg_native(params, bufs, P, n, ld, w, mask, outs)
        with self.lock:
            self.calls += 1
            off = 0
            for i in range(self.size):
                b = bufs[i]
                if P[i] == 0:
                    b.zero_()
                else:
                    rows = params[i].view(-1)[: P[i] * ld[i]].view(P[i], ld[i])[:, :n]
                    wt = torch.as_tensor(w[off : off + P[i]], dtype=torch.float32, device=rows.device)
                    b[:n].copy_((wt[:, None] * rows).sum(0))
                    b[n] = float(np.sum(w[off : off + P[i]], dtype=np.float64))
                off += P[i]
            self._reduce_apply(params, bufs, outs, P, n, ld, mask)

    def _reduce_apply(self, params, bufs, outs, P, n, ld, mask) -> None:
        if outs is None:
            res = list(bufs)
        else:
            for o, b in zip(outs, bufs):
                o[: n + 1].copy_(b[: n + 1])
            res = list(outs)
        self.all_reduce_([r[: n + 1] for r in res])
        off = 0
        for i in range(self.size):
            if P[i] > 0:
                b = res[i]
                mean = b[:n] / b[n].clamp_min(1e-30)
                rows = params[i].view(-1)[: P[i] * ld[i]].view(P[i], ld[i])
                for p in range(P[i]):
                    if mask[off + p] != 0:
                        rows[p, :n].copy_(mean)
            off += P[i]

    def fedavg_retry(self, params, bufs, outs, P, n, ld, mask) -> None:
        self._live()
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        with self.lock:
            self.calls += 1
            if all(t.is_cuda for t in params):
                self._native_reduce_apply(params, bufs, outs, P, n, ld, mask)
            else:
                self._reduce_apply(params, bufs, outs, P, n, ld, mask)

    def _fedavg_native(self, params, bufs, P, n, ld, w, mask, outs=None) -> None:
        """GPU members (a virtual mesh on one device): the same per-member reduce / apply launches
        as ``rmesh_fedavg``, with the all-reduce as stream-ordered torch adds — so a one-GPU
        rehearsal issues the real path's launches (host cost per round is representative)."""
        from myfyp_amd import ops

        fast = ops.fast_lib()
        w = np.ascontiguousarray(w, dtype=np.float32)
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        with self.lock:
            self.calls += 1
            off = 0
            for i in range(self.size):
                with torch.cuda.device(bufs[i].device):
                    st = _stream_ptr(bufs[i].device)
                    if P[i] == 0:
                        bufs[i].zero_()
                    else:
                        ops.check(fast.myfyp_fedavg_stacked_reduce(bufs[i].data_ptr(), params[i].data_ptr(), int(P[i]), int(n), int(ld[i]),
                                                                   w[off:].ctypes.data, st), "fedavg_stacked_reduce")
                off += P[i]
            self._native_reduce_apply(params, bufs, outs, P, n, ld, mask)

    def _native_reduce_apply(self, params, bufs, outs, P, n, ld, mask) -> None:
        from myfyp_amd import ops

        fast = ops.fast_lib()
        if outs is None:
            res = list(bufs)
        else:
            for o, b in zip(outs, bufs):
                with torch.cuda.device(o.device):
                    o[: n + 1].copy_(b[: n + 1])
            res = list(outs)
        self.all_reduce_([b[: n + 1] for b in res])
        off = 0
        for i in range(self.size):
            if P[i] > 0:
                with torch.cuda.device(res[i].device):
                    ops.check(fast.myfyp_fedavg_stacked_apply(params[i].data_ptr(), res[i].data_ptr(), int(P[i]), int(n), int(ld[i]),
                                                              mask[off:].ctypes.data, _stream_ptr(res[i].device)), "fedavg_stacked_apply")
            off += P[i]

    # ------------------------------------------------------------------ bucketed FedAvg
    def fedavg_bucketed(self, params, keeps, outs, P, n, ld, w, mask, comm_streams, bucket, apply=True) -> None:
        """Same launches as ``rmesh_fedavg_bucketed`` for GPU members (a virtual mesh: the
        per-bucket all-reduce is a stream-ordered sum on member 0's comm stream); CPU members
        compute the same result synchronously."""
        self._live()
        w = np.ascontiguousarray(w, dtype=np.float32)
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        ranges = _bucket_ranges(n, bucket)
        with self.lock:
            self.calls += 1
            if not all(t.is_cuda for t in params):
                off = 0
                for i in range(self.size):
                    kb = keeps[i]
                    kb.zero_()
                    if P[i] > 0:
                        rows = params[i].view(-1)[: P[i] * ld[i]].view(P[i], ld[i])[:, :n]
                        wt = torch.as_tensor(w[off : off + P[i]], dtype=torch.float32, device=rows.device)
                        kb[4 : 4 + n].copy_((wt[:, None] * rows).sum(0))
                        kb[0] = float(np.sum(w[off : off + P[i]], dtype=np.float64))
                    off += P[i]
                acc = keeps[0][: n + 4].clone()
                for kb in keeps[1:]:
                    acc.add_(kb[: n + 4].to(acc.device))
                for o in outs:
                    o[: n + 4].copy_(acc.to(o.device))
                if apply:
                    self._apply4(params, outs, P, n, ld, mask)
                return
            from myfyp_amd import ops

            fast = ops.fast_lib()
            off = 0
            for i in range(self.size):
                dev = keeps[i].device
                cs = comm_streams[i]
                with torch.cuda.device(dev):
                    cs.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(cs):
                        if P[i] == 0:
                            keeps[i].zero_()
                        else:
                            kp, sp = keeps[i].data_ptr(), params[i].data_ptr()
                            for k, (b0, b1) in enumerate(ranges):
                                ops.check(fast.myfyp_fedavg_bucket_reduce(kp + 4 * (4 + b0), kp if k == 0 else None, sp + 4 * b0, int(P[i]), b1 - b0, int(ld[i]),
                                                                          w[off:].ctypes.data, cs.cuda_stream), "fedavg_bucket_reduce")
                off += P[i]
            c0 = comm_streams[0]
            self._bucket_events = []
            for k, (b0, b1) in enumerate(ranges):
                lo, hi = (0 if k == 0 else 4 + b0), 4 + b1
                with torch.cuda.device(keeps[0].device):
                    for cs in comm_streams[1:]:
                        c0.wait_stream(cs)
                    with torch.cuda.stream(c0):
                        acc = keeps[0][lo:hi].clone()
                        for kb in keeps[1:]:
                            acc.add_(kb[lo:hi].to(acc.device))
                        for o in outs:
                            o[lo:hi].copy_(acc.to(o.device))
                    ev = torch.cuda.Event()
                    ev.record(c0)
                self._bucket_events.append(ev)
            for cs in comm_streams[1:]:
                cs.wait_event(self._bucket_events[-1])
            if not apply:
                return
            off = 0
            for i in range(self.size):
                if P[i] > 0 and np.any(mask[off : off + P[i]] != 0):
                    dev = outs[i].device
                    with torch.cuda.device(dev):
                        cur = torch.cuda.current_stream(dev)
                        op, dp = outs[i].data_ptr(), params[i].data_ptr()
                        for k, (b0, b1) in enumerate(ranges):
                            cur.wait_event(self._bucket_events[k])
                            ops.check(fast.myfyp_fedavg_bucket_apply(dp + 4 * b0, op + 4 * (4 + b0), op, int(P[i]), b1 - b0, int(ld[i]),
                                                                     mask[off:].ctypes.data, cur.cuda_stream), "fedavg_bucket_apply")
                off += P[i]

    def _apply4(self, params, outs, P, n, ld, mask) -> None:
        off = 0
        for i in range(self.size):
            if P[i] > 0:
                o = outs[i]
                mean = o[4 : 4 + n] / o[0].clamp_min(1e-12)
                rows = params[i].view(-1)[: P[i] * ld[i]].view(P[i], ld[i])
                for p in range(P[i]):
                    if mask[off + p] != 0:
                        rows[p, :n].copy_(mean)
            off += P[i]

    def delayed_land(self, params, snaps, outs, P, n, ld, ld_snap, mask, have_avg) -> None:
        self._live()
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        with self.lock:
            self.calls += 1
            off = 0
            for i in range(self.size):
                if P[i] > 0 and np.any(mask[off : off + P[i]] != 0):
                    dev = params[i].device
                    if params[i].is_cuda:
                        from myfyp_amd import ops

                        with torch.cuda.device(dev):
                            cur = torch.cuda.current_stream(dev)
                            if have_avg:
                                evs = getattr(self, "_bucket_events", None)
                                if not evs:
                                    raise MeshError("delayed_land: no bucketed exchange pending")
                                cur.wait_event(evs[-1])
                            o = outs[i]
                            ops.check(ops.fast_lib().myfyp_fedavg_delayed_land(params[i].data_ptr(), snaps[i].data_ptr(), int(ld_snap),
                                                                               o.data_ptr() + 16 if have_avg else None, o.data_ptr() if have_avg else None,
                                                                               int(P[i]), int(n), int(ld[i]), mask[off:].ctypes.data, cur.cuda_stream),
                                      "fedavg_delayed_land")
                    else:
                        rows = params[i].view(-1)[: P[i] * ld[i]].view(P[i], ld[i])
                        sn = snaps[i].view(-1)[: P[i] * ld_snap].view(P[i], ld_snap)
                        for p in range(P[i]):
                            if mask[off + p] != 0:
                                if have_avg:
                                    rows[p, :n] += outs[i][4 : 4 + n] / outs[i][0].clamp_min(1e-12) - sn[p, :n]
                                sn[p, :n].copy_(rows[p, :n])
                off += P[i]

    def fedavg_bucketed_retry(self, params, keeps, outs, P, n, ld, mask, apply=True) -> None:
        self._live()
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        with self.lock:
            self.calls += 1
            for o, kb in zip(outs, keeps):
                o[: n + 4].copy_(kb[: n + 4])
            self.all_reduce_([o[: n + 4] for o in outs])
            if not apply:
                self._bucket_events = [] if not params or not params[0].is_cuda else [torch.cuda.Event()]
                if self._bucket_events:
                    with torch.cuda.device(params[0].device):
                        self._bucket_events[0].record(torch.cuda.current_stream(params[0].device))
                return
            if all(t.is_cuda for t in params):
                from myfyp_amd import ops

                fast = ops.fast_lib()
                off = 0
                for i in range(self.size):
                    if P[i] > 0:
                        with torch.cuda.device(outs[i].device):
                            op = outs[i].data_ptr()
                            ops.check(fast.myfyp_fedavg_bucket_apply(params[i].data_ptr(), op + 16, op, int(P[i]), int(n), int(ld[i]), mask[off:].ctypes.data,
                                                                     _stream_ptr(outs[i].device)), "fedavg_bucket_apply")
                    off += P[i]
            else:
                self._apply4(params, outs, P, n, ld, mask)

    def shrink(self, keep) -> None:
        with self.lock:
            self.devices = [self.devices[k] for k in keep]
            self._stalled = {keep.index(r) for r in self._stalled if r in keep} if self._stalled else set()
            self._injected = None
            self.aborted = False
            self.shrinks += 1


class RcclMesh(DeviceMesh):
    """``csrc/runtime/rccl_mesh.hip`` through ctypes (GIL held: every call only enqueues)."""

    kind = "rccl"

    def __init__(self, devices: Sequence[torch.device]) -> None:
        super().__init__(devices)
        from myfyp_amd.ops import _native

        _native.load(required=True)
        lib = ctypes.PyDLL(_native.LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        self._lib = lib
        idx = [d.index if d.index is not None else 0 for d in self.devices]
        if len(set(idx)) != len(idx):
            raise ValueError(f"RcclMesh: every device at most once (got {idx}); use HostMesh for virtual members")
        arr = (ctypes.c_int * len(idx))(*idx)
        self._h = lib.rmesh_create(len(idx), arr)
        if not self._h:
            raise MeshError(f"ncclCommInitAll over devices {idx} failed: {self._err()}")

    def _err(self) -> str:
        return self._lib.rmesh_last_error().decode()

    def _rc(self, rc: int, what: str) -> None:
        if rc != 0:
            raise MeshError(f"{what}: {self._err()}")

    def _streams(self) -> ctypes.Array:
        return _ptrs([_stream_ptr(d) for d in self.devices])

    @staticmethod
    def _dtype(t: torch.Tensor) -> int:
        code = _DTYPE.get(t.dtype)
        if code is None:
            raise TypeError(f"mesh collectives: unsupported dtype {t.dtype}")
        return code

    def all_reduce_(self, ts, op: str = "sum") -> None:
        self._check_members(ts, "all_reduce")
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_allreduce(self._h, _ptrs([t.data_ptr() for t in ts]), ts[0].numel(), self._dtype(ts[0]), _OPS[op], self._streams()),
                     "rmesh_allreduce")

    def broadcast_(self, ts, root: int) -> None:
        self._check_members(ts, "broadcast")
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_broadcast(self._h, _ptrs([t.data_ptr() for t in ts]), ts[0].numel(), self._dtype(ts[0]), int(root), self._streams()),
                     "rmesh_broadcast")

    def all_gather_(self, outs, ins) -> None:
        self._check_members(ins, "all_gather")
        self._check_members(outs, "all_gather")
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_allgather(self._h, _ptrs([t.data_ptr() for t in ins]), _ptrs([t.data_ptr() for t in outs]), ins[0].numel(),
                                               self._dtype(ins[0]), self._streams()), "rmesh_allgather")

    def p2p_(self, ops) -> None:
        if not ops:
            return
        kinds = (ctypes.c_int * len(ops))(*[0 if k == "send" else 1 for k, _, _, _ in ops])
        ranks = (ctypes.c_int * len(ops))(*[r for _, r, _, _ in ops])
        peers = (ctypes.c_int * len(ops))(*[p for _, _, p, _ in ops])
        counts = (ctypes.c_int64 * len(ops))(*[t.numel() for _, _, _, t in ops])
        dt = self._dtype(ops[0][3])
        if any(self._dtype(t) != dt for _, _, _, t in ops):
            raise TypeError("p2p: one dtype per exchange")
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_p2p(self._h, len(ops), kinds, ranks, peers, _ptrs([t.data_ptr() for _, _, _, t in ops]), counts, dt,
                                         _ptrs([_stream_ptr(self.devices[r]) for _, r, _, _ in ops])), "rmesh_p2p")

    def fedavg_stacked(self, params, bufs, P, n, ld, w, mask, outs=None) -> None:
        w = np.ascontiguousarray(w, dtype=np.float32)
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        Pa = (ctypes.c_int * self.size)(*[int(p) for p in P])
        lda = (ctypes.c_int64 * self.size)(*[int(x) for x in ld])
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_fedavg(self._h, _ptrs([t.data_ptr() for t in params]), _ptrs([t.data_ptr() for t in bufs]), Pa, int(n), lda,
                                            w.ctypes.data, mask.ctypes.data, self._streams(),
                                            None if outs is None else _ptrs([t.data_ptr() for t in outs])), "rmesh_fedavg")

    def fedavg_retry(self, params, bufs, outs, P, n, ld, mask) -> None:
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        Pa = (ctypes.c_int * self.size)(*[int(p) for p in P])
        lda = (ctypes.c_int64 * self.size)(*[int(x) for x in ld])
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_fedavg_retry(self._h, _ptrs([t.data_ptr() for t in params]), _ptrs([t.data_ptr() for t in bufs]),
                                                  _ptrs([t.data_ptr() for t in outs]), Pa, int(n), lda, mask.ctypes.data, self._streams()),
                     "rmesh_fedavg_retry")

    def fedavg_bucketed(self, params, keeps, outs, P, n, ld, w, mask, comm_streams, bucket, apply=True) -> None:
        w = np.ascontiguousarray(w, dtype=np.float32)
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        Pa = (ctypes.c_int * self.size)(*[int(p) for p in P])
        lda = (ctypes.c_int64 * self.size)(*[int(x) for x in ld])
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_fedavg_bucketed(self._h, _ptrs([t.data_ptr() for t in params]), _ptrs([t.data_ptr() for t in keeps]),
                                                     _ptrs([t.data_ptr() for t in outs]), Pa, int(n), lda, w.ctypes.data, mask.ctypes.data, self._streams(),
                                                     _ptrs([s.cuda_stream for s in comm_streams]), int(bucket), int(bool(apply))), "rmesh_fedavg_bucketed")

    def delayed_land(self, params, snaps, outs, P, n, ld, ld_snap, mask, have_avg) -> None:
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        Pa = (ctypes.c_int * self.size)(*[int(p) for p in P])
        lda = (ctypes.c_int64 * self.size)(*[int(x) for x in ld])
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_delayed_land(self._h, _ptrs([t.data_ptr() for t in params]), _ptrs([t.data_ptr() for t in snaps]),
                                                  _ptrs([t.data_ptr() for t in outs]), Pa, int(n), lda, int(ld_snap), mask.ctypes.data, self._streams(),
                                                  int(bool(have_avg))), "rmesh_delayed_land")

    def fedavg_bucketed_retry(self, params, keeps, outs, P, n, ld, mask, apply=True) -> None:
        mask = np.ascontiguousarray(mask, dtype=np.float32)
        Pa = (ctypes.c_int * self.size)(*[int(p) for p in P])
        lda = (ctypes.c_int64 * self.size)(*[int(x) for x in ld])
        with self.lock:
            self.calls += 1
            self._rc(self._lib.rmesh_fedavg_bucketed_retry(self._h, _ptrs([t.data_ptr() for t in params]), _ptrs([t.data_ptr() for t in keeps]),
                                                           _ptrs([t.data_ptr() for t in outs]), Pa, int(n), lda, mask.ctypes.data, self._streams(),
                                                           int(bool(apply))), "rmesh_fedavg_bucketed_retry")

    def inject_error(self, rank: int) -> None:
        with self.lock:
            self._rc(self._lib.rmesh_debug_inject(self._h, int(rank)), "rmesh_debug_inject")

    def check(self) -> None:
        with self.lock:
            self._rc(self._lib.rmesh_check(self._h), "rmesh_check")

    def abort(self) -> None:
        with self.lock:
            self._rc(self._lib.rmesh_abort(self._h), "rmesh_abort")

    def shrink(self, keep) -> None:
        arr = (ctypes.c_int * len(keep))(*[int(k) for k in keep])
        with self.lock:
            self._rc(self._lib.rmesh_shrink(self._h, arr, len(keep)), "rmesh_shrink")
            self.devices = [self.devices[k] for k in keep]
            self.shrinks += 1

    def rebuild(self, keep) -> None:
        arr = (ctypes.c_int * len(keep))(*[int(k) for k in keep])
        with self.lock:
            self._rc(self._lib.rmesh_rebuild(self._h, arr, len(keep)), "rmesh_rebuild")
            self.devices = [self.devices[k] for k in keep]
            self.shrinks += 1

    def close(self) -> None:
        with self.lock:
            if self._h:
                self._lib.rmesh_destroy(self._h)
                self._h = None


def make_mesh(devices: Sequence[torch.device], backend: Optional[str] = None) -> DeviceMesh:
    """``backend``: "rccl", "host" or None (RCCL when every member is a distinct GPU)."""
    devs = [torch.device(d) for d in devices]
    if backend is None:
        distinct = len({(d.type, d.index) for d in devs}) == len(devs)
        backend = "rccl" if all(d.type == "cuda" for d in devs) and distinct else "host"
    if backend == "rccl":
        return RcclMesh(devs)
    if backend == "host":
        return HostMesh(devs)
    raise ValueError(f"unknown mesh backend {backend!r}")
