"""Failure handling of the in-process device mesh: a deadline and an asynchronous-error watch on
every mesh collective, abort, rebuild over the responsive devices, and a re-run of the round's
FedAvg over what arrived.

Reference semantics. The reference aggregator waits for the trainers' models and, when
``AGGREGATION_TIMEOUT`` expires, aggregates whatever arrived
(``p2pfl/learning/aggregators/aggregator.py:177-208``); non-trainers give up on the same timeout
(``p2pfl/stages/base_node/wait_agg_models_stage.py:40-67``). In the mesh a peer's model "arrives"
when its device completes the round's epoch and joins the grouped all-reduce. A device that never
gets there holds every other device's RCCL kernel, so the guard is what turns "wait for the
models" into "wait until the deadline, then aggregate the ones that arrived" (SURVEY §5.3, §7.4.3):

* :meth:`MeshGuard.track` — after a collective has been enqueued, one completion marker per member
  device (an event on that device's stream) and a deadline (``Settings.COLLECTIVE_TIMEOUT``) are
  registered, with an optional ``retry`` that re-runs the collective from retained inputs;
* a watchdog thread polls the pending collectives every 20 ms: ``rmesh_check``
  (``ncclCommGetAsyncError``) and the deadline. On an error or an expired deadline it aborts the
  mesh (``ncclCommAbort`` on every communicator): RCCL kernels stuck on a dead device end, so the
  survivors' streams drain;
* :meth:`MeshGuard.confirm` runs on the round driver at the next weights section, while the next
  local epoch (already queued behind the collective) runs, like the ranks path's deferred
  confirmation (``Federation.confirm_collectives``). On a failure it aborts (if the watchdog has
  not), probes every member device with a fresh marker (bounded by ``Settings.FAILURE_TIMEOUT``),
  rebuilds the mesh over the devices that answered (``rmesh_shrink``), stops the peers of the
  devices that did not, and re-runs each pending collective's ``retry`` over the survivors: FedAvg
  all-reduces the retained per-device partial sums again and re-applies the mean. As on the ranks
  path, the local epoch that started from the failed round's rows is discarded: every survivor
  continues from the same survivors' average of the failed round.

A collective without a ``retry`` (broadcast of the initial model, neighbour exchange, SCAFFOLD,
FedMedian) is detected, aborted and rebuilt the same way; its result on the survivors is whatever
landed before the abort, and a warning says so.
"""

from __future__ import annotations

import threading
import time
from typing import Callable, List, Optional

from myfyp_amd.management.logger import logger
from myfyp_amd.parallel.device_mesh import MeshError
from myfyp_amd.settings import Settings


class MeshOp:
    """One enqueued mesh collective awaiting confirmation."""

    def __init__(self, kind: str, members: List[int], markers: list, retry: Optional[Callable[[], None]], timeout: float) -> None:
        self.kind = kind
        self.members = list(members)  # original mesh ranks at issue time
        self.markers = markers
        self.retry = retry
        self.t0 = time.perf_counter()
        self.deadline = self.t0 + timeout

    def done(self) -> bool:
        return all(m.query() for m in self.markers)


class MeshGuard:
    """See the module docstring. One per :class:`~myfyp_amd.parallel.federation.Federation` with a mesh."""

    def __init__(self, fed) -> None:
        self.fed = fed
        self.pending: List[MeshOp] = []
        self.lock = threading.RLock()
        self.failure: Optional[str] = None  # set by the watchdog (or confirm) on an error / deadline
        self.aborted = False
        self.recoveries = 0
        self.lost: List[int] = []  # mesh ranks dropped as unresponsive
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    # ------------------------------------------------------------------ registration
    @property
    def mesh(self):
        return self.fed.mesh

    def _timeout(self) -> float:
        return float(Settings.COLLECTIVE_TIMEOUT)

    def track(self, kind: str, retry: Optional[Callable[[], None]] = None, streams=None) -> None:
        """Register the collective just enqueued on every member's current stream (or on
        ``streams[i]``: a delayed exchange that no compute stream waits on)."""
        if not Settings.COLLECTIVE_FAILOVER or self.mesh is None:
            return
        markers = [self.mesh.marker(i, None if streams is None else streams[i]) for i in range(self.mesh.size)]
        with self.lock:
            self.pending.append(MeshOp(kind, self.fed.mesh_members, markers, retry, self._timeout()))
        self._ensure_thread()

    def _ensure_thread(self) -> None:
        if self._thread is None:
            self._thread = threading.Thread(target=self._watch, name="mesh-watchdog", daemon=True)
            self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        t = self._thread
        if t is not None and t is not threading.current_thread():
            t.join(timeout=2.0)
        self._thread = None

    # ------------------------------------------------------------------ watchdog
    def _error(self) -> Optional[str]:
        try:
            self.mesh.check()
            return None
        except MeshError as e:
            return str(e)

    def _watch(self) -> None:
        while not self._stop.wait(0.02):
            with self.lock:
                if not self.pending or self.aborted or self.mesh is None:
                    continue
                err = self._error()
                op = self.pending[0]
                expired = time.perf_counter() > op.deadline and not op.done()
                if err is None and not expired:
                    continue
                reason = err or f"{op.kind}: not complete on every device after {self._timeout():.1f} s"
                self._abort(reason)

    def _abort(self, reason: str) -> None:
        if self.aborted:
            return
        self.failure = reason
        logger.warning("rank0", f"mesh watchdog: {reason}; aborting the mesh (ncclCommAbort)")
        try:
            self.mesh.abort()
        except MeshError as e:  # best effort: the mesh is rebuilt next
            logger.warning("rank0", f"mesh abort: {e}")
        self.aborted = True

    # ------------------------------------------------------------------ confirmation
    def confirm(self) -> bool:
        """Confirm every pending collective (round driver, next weights section / shutdown).
        Returns True if a recovery ran."""
        if self.mesh is None:
            return False
        recovered = False
        for _ in range(max(2, self.mesh.size + 1)):
            failed = self._wait_pending()
            if failed is None:
                return recovered
            self._recover(failed)
            recovered = True
        raise MeshError("mesh collectives failed again after repeated recoveries")

    def _wait_pending(self) -> Optional[str]:
        spin = 0
        while True:
            with self.lock:
                if self.failure is not None or self.aborted:
                    return self.failure or "mesh aborted"
                if not self.pending:
                    err = self._error()
                    return err
                op = self.pending[0]
                if op.done():
                    err = self._error()
                    if err is not None:
                        return err
                    self.pending.pop(0)
                    continue
                if time.perf_counter() > op.deadline:
                    return f"{op.kind}: not complete on every device after {self._timeout():.1f} s"
            spin += 1
            time.sleep(0 if spin < 200 else 0.0005)

    def _probe(self) -> List[int]:
        """Mesh ranks (original numbering) whose device completes a fresh marker within
        ``FAILURE_TIMEOUT`` (the markers go behind everything queued, stuck work included)."""
        members = list(self.fed.mesh_members)
        marks = [self.mesh.marker(i) for i in range(self.mesh.size)]
        deadline = time.perf_counter() + float(Settings.FAILURE_TIMEOUT)
        ok = [False] * len(marks)
        while True:
            for i, m in enumerate(marks):
                ok[i] = ok[i] or m.query()
            if all(ok) or time.perf_counter() > deadline:
                break
            time.sleep(0.001)
        return [r for r, good in zip(members, ok) if good]

    def _recover(self, reason: str) -> None:
        with self.lock:
            self._abort(reason)
            ops = list(self.pending)
            self.pending.clear()
        alive = self._probe()
        if not alive:
            raise MeshError(f"mesh recovery: no device responded ({reason})")
        lost = [r for r in self.fed.mesh_members if r not in alive]
        keep = [i for i, r in enumerate(self.fed.mesh_members) if r in alive]
        t0 = time.perf_counter()
        self.mesh.shrink(keep)  # the communicators are aborted: fresh init-all over the survivors
        self.fed.mesh_members = [self.fed.mesh_members[i] for i in keep]
        with self.lock:
            self.aborted = False
            self.failure = None
        self.recoveries += 1
        self.lost += lost
        self.fed.record("mesh_recovery", time.perf_counter() - t0)
        logger.warning("rank0", f"mesh recovered from '{reason}': devices {lost} dropped, continuing over mesh ranks {self.fed.mesh_members}")
        if lost:
            self.fed.mesh_drop_ranks(lost)
        for op in ops:
            if op.retry is None:
                logger.warning("rank0", f"mesh {op.kind}: no retained inputs; survivors keep what landed before the abort")
                continue
            op.retry()  # over the current (rebuilt) mesh members
            self.track(op.kind if op.kind.endswith("(retry)") else f"{op.kind} (retry)", op.retry)
