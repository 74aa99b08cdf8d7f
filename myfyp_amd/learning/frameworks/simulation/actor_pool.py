"""Device pool: simulated peers time-multiplexed onto the host's GPUs.

Parity target: ``p2pfl/learning/frameworks/simulation/actor_pool.py:39-357`` (``VirtualLearnerActor``
``:39-66``, singleton ``SuperActorPool`` ``:69-357``: idle/pending bookkeeping, per-address futures,
dead-actor flagging and removal, pool shrinking when resources go away).

The reference runs each virtual client in a Ray actor process and, every round, pickles the whole
learner — model AND dataset — into it. On an MI355X node that is the wrong shape:
one process per GPU already owns the device, and 288 GB of HBM holds every simulated peer's model
and data resident. So here a pool worker ("actor") is a thread of this process bound to ONE device
and owning ONE HIP stream; a job runs the learner in place on that stream (nothing is serialised,
tensors never leave HBM) and synchronises the stream before its result is published. V virtual
peers share G devices through ``num_gpus``-fractional workers (0.25 → four streams per GPU), and a
peer is pinned to one device by :meth:`SuperActorPool.place` so its tensors stay where they are;
jobs prefer an idle worker on the peer's device.

Failure model: a job that raises an ordinary exception fails only that job. A job that hits a
device-fatal HIP error (illegal address, launch failure, ECC ...) kills its worker: the job fails
with :class:`ActorDiedError`, the worker is flagged and removed from the pool, queued jobs move on to
the surviving workers, and when no worker is left the remaining jobs fail instead of hanging.
"""

from __future__ import annotations

import contextlib
import itertools
import queue
import threading
import time
from collections import Counter, deque
from concurrent.futures import FIRST_COMPLETED, Future, wait
from typing import Any, Callable, Deque, Dict, List, Optional, Set, Tuple

from myfyp_amd.learning.frameworks.simulation.utils import (
    Resources,
    check_client_resources,
    pool_devices,
    pool_size_from_resources,
)
from myfyp_amd.management.logger import logger

# substrings of HIP runtime errors after which the device context is unusable
_FATAL_MARKERS = (
    "illegal memory access",
    "illegal address",
    "unspecified launch failure",
    "hipErrorLaunchFailure",
    "hipErrorIllegalAddress",
    "device-side assert",
    "uncorrectable ECC",
    "hipErrorNoDevice",
    "HSA_STATUS_ERROR",
)


class ActorDiedError(RuntimeError):
    """A pool worker is gone (its device context failed or it was terminated)."""

    def __init__(self, actor_id: str, cause: Optional[BaseException] = None) -> None:
        super().__init__(f"Actor({actor_id}) died" + (f": {cause}" if cause is not None else ""))
        self.actor_id = actor_id
        self.cause = cause


def _is_fatal(e: BaseException) -> bool:
    if isinstance(e, ActorDiedError):
        return True
    msg = str(e)
    return any(m in msg for m in _FATAL_MARKERS)


class VirtualLearnerActor:
    """One pool worker: a daemon thread bound to ``device`` with its own HIP stream (parity:
    ``actor_pool.py:39-66``). ``execute(fn, *args)`` runs ``fn(actor, *args)`` on the worker and
    returns a :class:`concurrent.futures.Future`; ``fit``/``evaluate`` are the job bodies."""

    _ids = itertools.count()

    def __init__(self, device: str = "cpu") -> None:
        import torch

        self.actor_id = f"actor-{next(self._ids)}"
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", 0)
        self._jobs: "queue.SimpleQueue[Optional[Tuple[Future, Callable, tuple]]]" = queue.SimpleQueue()
        self._alive = True
        self._stream = None
        self.jobs_done = 0
        self._thread = threading.Thread(target=self._loop, name=f"{self.actor_id}@{self.device}", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ job bodies
    def fit(self, addr: str, learner: Any) -> Tuple[str, Any]:
        """Train ``learner`` in place; returns ``(addr, model)``."""
        return addr, learner.fit()

    def evaluate(self, addr: str, learner: Any) -> Tuple[str, Dict[str, float]]:
        return addr, learner.evaluate()

    # ------------------------------------------------------------------ worker
    @property
    def alive(self) -> bool:
        return self._alive

    @property
    def device_key(self) -> str:
        return str(self.device)

    def execute(self, fn: Callable[..., Any], *args: Any) -> Future:
        fut: Future = Future()
        if not self._alive:
            fut.set_exception(ActorDiedError(self.actor_id))
            return fut
        self._jobs.put((fut, fn, args))
        return fut

    def terminate(self) -> None:
        """Stop after the queued jobs (parity: ``VirtualLearnerActor.terminate``)."""
        self._jobs.put(None)

    def join(self, timeout: Optional[float] = None) -> None:
        self._thread.join(timeout)

    def _context(self) -> contextlib.ExitStack:
        stack = contextlib.ExitStack()
        if self.device.type == "cuda":
            import torch

            stack.enter_context(torch.cuda.device(self.device))
            if self._stream is None:
                self._stream = torch.cuda.Stream(self.device)
            stack.enter_context(torch.cuda.stream(self._stream))
        return stack

    def _loop(self) -> None:
        while True:
            item = self._jobs.get()
            if item is None:
                break
            fut, fn, args = item
            if not fut.set_running_or_notify_cancel():
                continue
            try:
                with self._context():
                    res = fn(self, *args)
                    if self._stream is not None:
                        self._stream.synchronize()  # the result is complete before anyone reads it
            except BaseException as e:  # noqa: BLE001 - every failure is reported through the future
                if _is_fatal(e):
                    self._alive = False
                    fut.set_exception(e if isinstance(e, ActorDiedError) else ActorDiedError(self.actor_id, e))
                    break
                fut.set_exception(e)
            else:
                self.jobs_done += 1
                fut.set_result(res)
        self._alive = False
        while True:  # jobs queued behind a death or a terminate never run
            try:
                item = self._jobs.get_nowait()
            except queue.Empty:
                break
            if item is not None and item[0].set_running_or_notify_cancel():
                item[0].set_exception(ActorDiedError(self.actor_id))


class SuperActorPool:
    """Process-wide singleton pool of device workers (parity: ``actor_pool.py:69-357``)."""

    _instance: Optional["SuperActorPool"] = None
    _instance_lock = threading.Lock()

    def __new__(cls, *args: Any, **kwargs: Any) -> "SuperActorPool":
        with cls._instance_lock:
            if cls._instance is None:
                cls._instance = super().__new__(cls)
            return cls._instance

    def __init__(self, resources: Optional[Resources] = None, actor_list: Optional[List[VirtualLearnerActor]] = None, inventory: Optional[Dict[str, int]] = None) -> None:
        if getattr(self, "initialized", False):  # singleton: later constructions are lookups
            return
        self.lock = threading.RLock()
        self._cv = threading.Condition(self.lock)
        self._inventory = inventory
        self.resources = check_client_resources(resources)
        if actor_list is None:
            n = pool_size_from_resources(self.resources, inventory)
            actors = [self.create_actor(d) for d in pool_devices(self.resources, n, inventory)]
        else:
            actors = list(actor_list)
        self._actors: Dict[str, VirtualLearnerActor] = {a.actor_id: a for a in actors}
        self._idle_actors: List[VirtualLearnerActor] = list(actors)
        self._pending_submits: Deque[Tuple[Callable, Tuple[str, Any]]] = deque()
        self._future_to_actor: Dict[Future, Tuple[int, VirtualLearnerActor, str]] = {}
        self._next_task_index = 0
        self._addr_to_future: Dict[str, Dict[str, Any]] = {}
        self.actor_to_remove: Set[str] = set()
        self.num_actors = len(actors)
        self._placement: Dict[str, str] = {}
        self._draining = False
        self.initialized = True
        logger.info("ActorPool", f"Initialized with {self.num_actors} actors on {sorted(Counter(a.device_key for a in actors).items())}")

    # ------------------------------------------------------------------ lifecycle
    @classmethod
    def reset(cls) -> None:
        """Terminate the workers and drop the singleton (tests, re-configuration)."""
        with cls._instance_lock:
            inst, cls._instance = cls._instance, None
        if inst is not None and getattr(inst, "initialized", False):
            inst.shutdown()

    def shutdown(self, timeout: float = 5.0) -> None:
        with self.lock:
            actors = list(self._actors.values())
        for a in actors:
            a.terminate()
        for a in actors:
            a.join(timeout)

    def create_actor(self, device: Optional[str] = None) -> VirtualLearnerActor:
        return VirtualLearnerActor(device or "cpu")

    def add_actor(self, num_actors: int, device: Optional[str] = None) -> None:
        """Grow the pool; new workers go to ``device`` or round-robin over the configured devices."""
        with self.lock:
            if device:
                devs = [device] * num_actors
            else:
                devs = pool_devices(self.resources, self.num_actors + num_actors, self._inventory)[self.num_actors :]
            for d in devs:
                a = self.create_actor(d)
                self._actors[a.actor_id] = a
                self._idle_actors.append(a)
            self.num_actors += num_actors
            logger.info("ActorPool", f"Created {num_actors} actors")
            self._drain_pending()

    # ------------------------------------------------------------------ placement
    def devices(self) -> List[str]:
        with self.lock:
            return sorted({a.device_key for a in self._actors.values()})

    def place(self, addr: str) -> str:
        """Pin a virtual peer to the least-loaded device of the pool (sticky per address)."""
        with self.lock:
            if addr not in self._placement:
                devs = self.devices() or ["cpu"]
                load = Counter(self._placement.values())
                self._placement[addr] = min(devs, key=lambda d: (load[d], d))
            return self._placement[addr]

    @staticmethod
    def _job_device(learner: Any) -> Optional[str]:
        dev = getattr(learner, "device", None)
        if dev is None:
            return None
        s = str(dev)
        return "cuda:0" if s == "cuda" else s

    def _pick_idle(self, device: Optional[str]) -> Optional[VirtualLearnerActor]:
        for i in range(len(self._idle_actors) - 1, -1, -1):
            if device is None or self._idle_actors[i].device_key == device:
                return self._idle_actors.pop(i)
        if self._idle_actors and not any(a.device_key == device for a in self._actors.values()):
            return self._idle_actors.pop()  # no worker on that device at all: any one will do
        return None

    # ------------------------------------------------------------------ submission
    def submit(self, fn: Callable[..., Any], value: Tuple[str, Any]) -> bool:
        """Start ``fn(actor, addr, learner)`` on an idle worker suited to the learner's device.
        Returns False (job left for later) when none is idle."""
        addr, learner = value
        with self.lock:
            while True:
                actor = self._pick_idle(self._job_device(learner))
                if actor is None:
                    return False
                if self._check_and_remove_actor_from_pool(actor):
                    break
            fut = actor.execute(fn, addr, learner)
            self._future_to_actor[fut] = (self._next_task_index, actor, addr)
            self._next_task_index += 1
            self._addr_to_future.setdefault(addr, {})["future"] = fut
        fut.add_done_callback(self._on_done)
        return True

    def submit_learner_job(self, actor_fn: Callable[..., Any], job: Tuple[str, Any]) -> None:
        """Submit now, or queue until a suitable worker frees up (parity: ``actor_pool.py:186-201``)."""
        addr, _ = job
        with self.lock:
            self._reset_addr_to_future_dict(addr)
            if not self.submit(actor_fn, job):
                self._pending_submits.append((actor_fn, job))
                self._drain_pending()  # fails the job at once if the pool has no live worker

    def _drain_pending(self) -> None:
        if self._draining:  # re-entered from a job that completed inside submit()
            return
        self._draining = True
        try:
            progress = True
            while progress and self._pending_submits:
                progress = False
                for _ in range(len(self._pending_submits)):
                    fn, job = self._pending_submits.popleft()
                    if self.submit(fn, job):
                        progress = True
                    else:
                        self._pending_submits.append((fn, job))
            if not self._actors:  # nobody left to run them
                while self._pending_submits:
                    _, (addr, _) = self._pending_submits.popleft()
                    self._fail_addr(addr, ActorDiedError("pool", RuntimeError("the pool has no live actors")))
        finally:
            self._draining = False

    def _fail_addr(self, addr: str, exc: BaseException) -> None:
        fut: Future = Future()
        fut.set_exception(exc)
        ent = self._addr_to_future.setdefault(addr, {})
        ent["future"] = fut
        ent["ready"] = True
        self._cv.notify_all()

    def _on_done(self, fut: Future) -> None:
        with self.lock:
            _, actor, addr = self._future_to_actor.pop(fut, (None, None, None))
            if actor is None:
                return
            exc = fut.exception()
            if isinstance(exc, ActorDiedError) or not actor.alive:
                self._flag_actor_for_removal(actor.actor_id)
                self._check_and_remove_actor_from_pool(actor)
            elif self._check_actor_fits_in_pool():
                if self._check_and_remove_actor_from_pool(actor):
                    self._idle_actors.append(actor)
            else:
                self._actors.pop(actor.actor_id, None)
                actor.terminate()
            if addr in self._addr_to_future and self._addr_to_future[addr].get("future") is fut:
                self._flag_future_as_ready(addr)
            self._drain_pending()
            self._cv.notify_all()

    # ------------------------------------------------------------------ futures per address
    def _flag_future_as_ready(self, addr: str) -> None:
        self._addr_to_future[addr]["ready"] = True

    def _reset_addr_to_future_dict(self, addr: str) -> None:
        ent = self._addr_to_future.setdefault(addr, {})
        ent["future"] = None
        ent["ready"] = False

    def _is_future_ready(self, addr: str) -> bool:
        if addr not in self._addr_to_future:
            logger.error("ActorPool", f"No job was submitted for {addr}")
            return False
        return bool(self._addr_to_future[addr]["ready"])

    def _fetch_future_result(self, addr: str) -> Tuple[str, Any]:
        fut = self._addr_to_future[addr]["future"]
        if fut is None:
            raise RuntimeError(f"ActorPool: no result pending for {addr}")
        try:
            res_addr, result = fut.result(timeout=0)
        except ActorDiedError as ex:
            if ex.actor_id in self._actors:
                self._flag_actor_for_removal(ex.actor_id)
            raise
        finally:
            self._reset_addr_to_future_dict(addr)
        assert res_addr == addr, (res_addr, addr)
        return res_addr, result

    # ------------------------------------------------------------------ pool membership
    def _flag_actor_for_removal(self, actor_id: str) -> None:
        with self.lock:
            self.actor_to_remove.add(actor_id)
            logger.debug("ActorPool", f"Actor({actor_id}) will be removed from pool.")

    def _check_and_remove_actor_from_pool(self, actor: VirtualLearnerActor) -> bool:
        """True if ``actor`` stays in the pool; a flagged (or dead) actor is removed."""
        with self.lock:
            if actor.actor_id in self.actor_to_remove or not actor.alive:
                self.actor_to_remove.discard(actor.actor_id)
                if self._actors.pop(actor.actor_id, None) is not None:
                    self.num_actors -= 1
                    logger.debug("ActorPool", f"REMOVED actor {actor.actor_id} from pool")
                actor.terminate()
                return False
            return True

    def _check_actor_fits_in_pool(self) -> bool:
        """Shrink by one worker when the host can no longer hold the current pool."""
        try:
            fits = pool_size_from_resources(self.resources, self._inventory)
        except ValueError:
            fits = 0
        if fits < self.num_actors:
            self.num_actors -= 1
            return False
        return True

    # ------------------------------------------------------------------ results
    def has_next(self) -> bool:
        with self.lock:
            return bool(self._future_to_actor or self._pending_submits)

    def process_unordered_future(self, timeout: Optional[float] = None) -> None:
        """Block until any running job finishes (its bookkeeping runs in the completion callback).
        Raises ``StopIteration`` with nothing in flight, ``TimeoutError`` on timeout."""
        with self.lock:
            running = list(self._future_to_actor)
            pending = bool(self._pending_submits)
        if not running:
            if pending:
                return
            raise StopIteration("No more results to get")
        done, _ = wait(running, timeout=timeout, return_when=FIRST_COMPLETED)
        if not done:
            raise TimeoutError("Timed out waiting for result")

    def get_learner_result(self, addr: str, timeout: Optional[float]) -> Tuple[str, Any]:
        """Wait for ``addr``'s job and return ``(addr, result)``; its exception is re-raised."""
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while not self._is_future_ready(addr):
                if addr not in self._addr_to_future or not (self._future_to_actor or self._pending_submits):
                    break
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    raise TimeoutError(f"Timed out waiting for the result of {addr}")
                self._cv.wait(left)
            return self._fetch_future_result(addr)
