"""Process-level federation runtime: one process per GPU, RCCL/xGMI weights plane.

The reference moves every model through gRPC + pickle between peers and reduces on the host with
NumPy. Here each process owns one GPU and hosts ``P`` co-located peers;
the peers of all processes form one federation:

* **control plane** — co-located peers talk over the in-process bus; peers on other ranks are
  reached through :class:`StoreBus`, a mailbox over the ``torch.distributed`` TCPStore (no extra
  dependency, works wherever ``torchrun`` works);
* **weights plane** — round-level collectives executed ONCE per process by a *gang* of the local
  peers' learning threads: votes are all-gathered so every rank computes the same train set; FedAvg
  is one weighted all-reduce (``n_i``-weighted local partial sum on the GPU → ``all_reduce(SUM)``
  over RCCL → scale → broadcast into every local peer's parameter row); the initial model is one
  broadcast from the initiator's rank;
* **fault tolerance** — a gang waits at most ``Settings.AGGREGATION_TIMEOUT`` for a co-located peer
  and then proceeds without it (the reference's "aggregate whatever arrived", ``aggregator.py:192-208``).
  Across ranks, every control-plane gather is also a liveness agreement (shared-memory membership
  protocol, ``csrc/host/shm_collective.cpp``): a rank whose last local peer stops mid-experiment
  *departs* (it never joins another collective), a rank whose heartbeat goes stale for
  ``Settings.FAILURE_TIMEOUT`` is evicted, and every survivor observes the same participant set at
  the same gather; before each weight collective the survivors re-agree and, on a change, rebuild
  their process groups over themselves (group-local rendezvous) — the reference's heartbeat
  eviction (``heartbeater.py:94-103``) for the RCCL weights plane;
* **in-flight failure** — a rank that dies *inside* a weight collective (after the pre-collective
  agreement) is caught by the collective guard: every wait on a weight collective polls the
  members' liveness (process gone / heartbeat stale, ``shmc_unresponsive``) and a watchdog thread
  aborts the device group (``ncclCommAbort`` through ``_abort_process_group``) so no survivor
  stays inside RCCL; the survivors agree on the outcome of every collective (one shared-memory
  gather) before anything is written, rebuild their groups over themselves and re-run the
  aggregation from the still-intact local rows (the reference's "aggregate whatever arrived",
  ``aggregator.py:191-208``, and drop-on-send-failure, ``grpc_client.py:176-186``);
* **device mesh** (``Federation.init(devices=G)``, ``Settings.MESH_DEVICES``, ``bench.py --gpus G``)
  — ONE process drives G GPUs, the reference's process model (all peers in one process,
  ``p2pfl/communication/protocols/memory/server_singleton.py:22-43``): peers are placed
  round-robin over the devices (:meth:`Federation.placement`), each device's peers form one stacked
  engine group, and the weights plane between devices is an in-process RCCL mesh
  (``ncclCommInitAll`` + grouped collectives from one thread, ``parallel/device_mesh.py`` /
  ``csrc/runtime/rccl_mesh.hip``). Votes, membership and agreement are plain function calls: there
  is no cross-process control plane. A device whose last peer stops leaves the mesh
  (``ncclCommAbort`` + ``ncclCommInitAll`` over the survivors);
* **forced collective** (``Settings.FORCE_COLLECTIVE`` / ``MYFYP_FORCE_COLLECTIVE=1``) — a
  single-process job still initialises the ``nccl`` (RCCL) process group at world size 1 and takes
  every multi-rank code path (bucketed side-stream FedAvg, broadcast, all-gather, group rebuild), so
  the RCCL data plane runs and can be profiled on one GPU.
"""

from __future__ import annotations

import contextlib
import datetime
import os
import sys
import pickle
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from myfyp_amd.management.logger import logger
from myfyp_amd.management.tracing import mark
from myfyp_amd.settings import Settings
from myfyp_amd.learning.frameworks.p2pfl_model import safe_loads
from myfyp_amd.utils.lockcheck import make_lock


# ---------------------------------------------------------------------------------------------
# communication statistics (node monitor: bytes moved, collective latency)
# ---------------------------------------------------------------------------------------------
class CommStats:
    """Bytes and latency per collective kind. Host-timed calls record wall time; device-timed
    ones (the side-stream FedAvg pipeline) record a pair of HIP events, resolved lazily when a
    snapshot is taken, so recording never waits on the GPU."""

    def __init__(self) -> None:
        self._lock = threading.Lock()
        self.bytes: Dict[str, int] = {}
        self.calls: Dict[str, int] = {}
        self.us_last: Dict[str, float] = {}
        self.us_total: Dict[str, float] = {}
        self._pending: List[tuple] = []

    def _add(self, kind: str, nbytes: int, us: Optional[float]) -> None:
        self.bytes[kind] = self.bytes.get(kind, 0) + int(nbytes)
        self.calls[kind] = self.calls.get(kind, 0) + 1
        if us is not None:
            self.us_last[kind] = us
            self.us_total[kind] = self.us_total.get(kind, 0.0) + us

    # device-timed kinds record their event pair once every TIME_EVERY calls: two timing events per
    # round sat on the critical-path FedAvg (~2.7 us each, profiles/r5_gap)
    TIME_EVERY = 16

    def timed(self, kind: str) -> bool:
        with self._lock:
            return self.calls.get(kind, 0) % self.TIME_EVERY == 0 or kind not in self.calls

    def host(self, kind: str, nbytes: int, seconds: float) -> None:
        with self._lock:
            self._add(kind, nbytes, seconds * 1e6)

    def device(self, kind: str, nbytes: int, ev0, ev1) -> None:
        with self._lock:
            if ev1 is None:  # an untimed call (sampled timing): bytes and count only
                self._add(kind, nbytes, None)
                return
            self._pending.append((kind, int(nbytes), ev0, ev1))
            if len(self._pending) > 256:  # never resolved (no snapshot taken): keep bytes, drop timing
                k, b, _, _ = self._pending.pop(0)
                self._add(k, b, None)

    def snapshot(self) -> Dict[str, Dict[str, float]]:
        with self._lock:
            keep = []
            for kind, nbytes, ev0, ev1 in self._pending:
                try:
                    done = ev1.query()
                except Exception:
                    done = True
                    ev0 = None
                if not done:
                    keep.append((kind, nbytes, ev0, ev1))
                    continue
                us = None
                if ev0 is not None:
                    try:
                        us = ev0.elapsed_time(ev1) * 1e3
                    except Exception:
                        us = None
                self._add(kind, nbytes, us)
            self._pending = keep
            return {k: {"bytes": self.bytes[k], "calls": self.calls[k], "us_last": self.us_last.get(k), "us_total": self.us_total.get(k, 0.0)}
                    for k in self.bytes}


# ---------------------------------------------------------------------------------------------
# cross-rank control bus
# ---------------------------------------------------------------------------------------------
class StoreBus:
    """Ordered per-rank mailboxes on a ``torch.distributed.Store``."""

    def __init__(self, store, rank: int, world: int, deliver: Callable[[str, str, dict], None]) -> None:
        self.store = store
        self.rank = rank
        self.world = world
        self._deliver = deliver
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._listen, name=f"storebus-{rank}", daemon=True)
        self._thread.start()

    def send(self, dest_rank: int, dest_addr: str, kind: str, msg: dict) -> None:
        seq = self.store.add(f"mbox/{dest_rank}/ctr", 1)
        self.store.set(f"mbox/{dest_rank}/{seq}", pickle.dumps((dest_addr, kind, msg)))

    def _listen(self) -> None:
        # non-blocking counter poll with adaptive back-off: control messages are rare (start/stop,
        # heartbeats), and a blocking store.wait() would pin the store socket at shutdown
        # after stop() one more pass delivers what is already queued (e.g. the relay's last metrics)
        seq = 1
        idle = 0.0005
        while True:
            try:
                ctr = self.store.add(f"mbox/{self.rank}/ctr", 0)
            except Exception:
                if self._stop.wait(0.05):
                    return
                continue
            if ctr < seq:
                if self._stop.is_set():
                    return
                self._stop.wait(idle)
                idle = min(idle * 2, 0.02)
                continue
            idle = 0.0005
            while seq <= ctr:
                key = f"mbox/{self.rank}/{seq}"
                try:
                    payload = self.store.get(key)
                    self.store.delete_key(key)
                except Exception:
                    break
                seq += 1
                try:
                    # the TCPStore is unauthenticated: decode with the restricted unpickler
                    dest, kind, msg = safe_loads(payload)
                    self._deliver(dest, kind, msg)
                except Exception as e:  # never kill the listener
                    logger.error(f"rank{self.rank}", f"StoreBus delivery failed: {e}")

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(timeout=2.0)


class RemotePeer:
    """Stub for a peer on another rank; quacks like a protocol for the in-memory client."""

    def __init__(self, fed: "Federation", rank: int, addr: str) -> None:
        self.fed, self.rank, self.addr = fed, rank, addr

    def is_running(self) -> bool:
        return True

    def handle_message(self, msg: dict) -> dict:
        self.fed.bus.send(self.rank, self.addr, "msg", msg)
        return {}

    def handle_weights(self, msg: dict) -> dict:
        self.fed.bus.send(self.rank, self.addr, "weights", msg)
        return {}

    def handshake(self, addr: str) -> bool:
        return True

    def remote_disconnect(self, addr: str) -> None:
        pass


# ---------------------------------------------------------------------------------------------
# local gang: one op at a time, executed once per process by the last arriving peer thread
# ---------------------------------------------------------------------------------------------
class LocalGang:
    """Barrier-with-payload across the co-located peers' learning threads."""

    def __init__(self) -> None:
        self._cv = threading.Condition()
        self._gen = 0
        self._arrived: Dict[str, Any] = {}
        self._result: Dict[int, Any] = {}
        self._error: Dict[int, BaseException] = {}

    def poke(self) -> None:
        """Membership changed (a peer left): let waiting members re-evaluate."""
        with self._cv:
            self._cv.notify_all()

    def run(self, member: str, members: Callable[[], List[str]], payload: Any, fn: Callable[[Dict[str, Any]], Any], timeout: float) -> Any:
        """``members`` is re-read on every wake-up so a peer that dies mid-round (fault injection,
        crash) stops being waited for as soon as it unregisters."""
        with self._cv:
            gen = self._gen
            self._arrived[member] = payload
            deadline = time.time() + timeout
            while gen == self._gen:
                live = members()
                if set(live).issubset(self._arrived) or time.time() >= deadline:
                    missing = set(live) - set(self._arrived)
                    if missing:
                        logger.warning(member, f"gang timeout; proceeding without {sorted(missing)}")
                    arrived, self._arrived = self._arrived, {}
                    self._gen += 1
                    self._cv.release()
                    try:
                        res, err = fn(arrived), None
                    except BaseException as e:
                        res, err = None, e
                    finally:
                        self._cv.acquire()
                    if err is not None:
                        self._error[gen] = err
                    else:
                        self._result[gen] = res
                    for old in [g for g in self._result if g < gen - 16]:
                        del self._result[old]
                    self._cv.notify_all()
                    break
                self._cv.wait(timeout=max(0.001, min(1.0, deadline - time.time())))
            while gen not in self._result and gen not in self._error:
                self._cv.wait(timeout=1.0)
            if gen in self._error:
                raise self._error[gen]
            return self._result[gen]


class MembershipChanged(RuntimeError):
    """A weight collective did not complete on every member (a rank died inside it). The groups
    have been rebuilt over the survivors; the aggregation must be re-run from its inputs."""


# ---------------------------------------------------------------------------------------------
# federation
# ---------------------------------------------------------------------------------------------
class Federation:
    """Singleton per process; created by :meth:`init`."""

    _instance: Optional["Federation"] = None

    def __init__(self, rank: int, world: int, local_rank: int, device: torch.device, store=None) -> None:
        self.rank, self.world, self.local_rank = rank, world, local_rank
        self.device = device
        self.store = store
        self.bus: Optional[StoreBus] = None
        self.central = None  # live metric relay to rank 0 (management/logger/central.py)
        self.comm = CommStats()
        self.local_nodes: Dict[str, Any] = {}
        self.local_order: List[str] = []
        self.peers: Dict[str, int] = {}  # addr -> rank (all peers, after finalize)
        self.gang = LocalGang()
        self.finalized = threading.Event()
        self.round_hooks: List[Callable[[int, "Federation"], None]] = []
        # called once per round and process when the round's train set is known, before its first
        # launch (the vote's gang leader, or the round driver): (round, federation)
        self.round_start_hooks: List[Callable[[int, "Federation"], None]] = []
        self.stats: Dict[str, List[float]] = {}
        self._lock = make_lock("Federation.state")
        self._cpu_pg = None
        self.shm = None  # node-local shared-memory control plane (single-node jobs)
        self._round_driver = None
        # membership (fault tolerance): live ranks, device group over them (None = WORLD)
        self.members: List[int] = list(range(world))
        self.departed = False
        self._pg = None
        self._hb_stop = threading.Event()
        self._hb_thread: Optional[threading.Thread] = None
        # collective data plane active: several ranks, or a forced single-rank RCCL group
        self.collective = world > 1
        self.forced = False
        # weights section (one aggregation): membership / departure frozen at entry
        self._section_lock = threading.RLock()
        self._frozen: Optional[Tuple[bool, List[int]]] = None
        self._depart_deferred = False
        # collective guard: watchdog state and the not-yet-confirmed device pipeline
        self._inflight: Optional[Tuple[Any, List[int]]] = None  # (group, members) of the running collective
        self._aborted: set = set()
        self._pending: List[Tuple[List[Any], List[int], Callable[[], None], Any]] = []
        self._wd_stop = threading.Event()
        self._wd_thread: Optional[threading.Thread] = None
        self.recoveries = 0
        # fault injection (fault_injection.crash_in_collective): called right before a weight
        # collective is issued, with its kind
        self.pre_collective_hooks: List[Callable[[str], None]] = []
        # in-process device mesh (parallel/device_mesh.py): the devices this process drives, the
        # mesh ranks still taking part (original numbering) and the round-robin placement cursor
        self.devices: List[torch.device] = [device]
        self.mesh = None
        self.mesh_guard = None  # parallel/mesh_guard.py (mesh runs)
        self.mesh_members: List[int] = [0]
        self._placed = 0
        self._mesh_scratch: Dict[Tuple[int, int], torch.Tensor] = {}

    # ------------------------------------------------------------------ lifecycle
    @classmethod
    def init(cls, backend: Optional[str] = None, devices: Any = None, mesh_backend: Optional[str] = None) -> "Federation":
        """Initialise from ``torchrun`` env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*), or — with
        ``devices`` (a count or a list of device strings; default ``Settings.MESH_DEVICES`` /
        ``MYFYP_MESH_DEVICES``) — as a single process driving a device mesh (env rank/world are then
        ignored: the process is the whole federation)."""
        if cls._instance is not None:
            return cls._instance
        if Settings.GIL_SWITCH_INTERVAL:
            sys.setswitchinterval(float(Settings.GIL_SWITCH_INTERVAL))
        if devices is None:
            env = os.environ.get("MYFYP_MESH_DEVICES", "")
            devices = int(env) if env.isdigit() else Settings.MESH_DEVICES
        devs = mesh_devices(devices)
        if devs is not None:
            return cls._init_mesh(devs, mesh_backend or Settings.MESH_BACKEND)
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
            device = torch.device("cuda", torch.cuda.current_device())
        else:
            device = torch.device("cpu")
        store = None
        forced = world == 1 and (bool(Settings.FORCE_COLLECTIVE) or os.environ.get("MYFYP_FORCE_COLLECTIVE", "0") not in ("", "0"))
        if forced:  # a one-rank RCCL job: rendezvous on this host
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket

                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if world > 1 or forced:
            import torch.distributed as dist

            if not dist.is_initialized():
                # MYFYP_DIST_BACKEND=gloo rehearses a multi-rank job on ONE GPU (RCCL refuses two
                # ranks on one device); production multi-GPU jobs use RCCL ("nccl")
                be = backend or os.environ.get("MYFYP_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
                kw = {"timeout": datetime.timedelta(seconds=Settings.COLLECTIVE_TIMEOUT)}
                if be == "nccl":
                    kw["device_id"] = device
                    # RCCL's channel cap (one workgroup per channel): the CUs an RCCL kernel can
                    # hold beside a persistent epoch (rccl_reserved_cus)
                    os.environ.setdefault("NCCL_MAX_NCHANNELS", str(int(Settings.RCCL_MAX_CHANNELS)))
                    os.environ.setdefault("NCCL_MAX_CTAS", os.environ["NCCL_MAX_NCHANNELS"])
                dist.init_process_group(backend=be, **kw)
            store = _default_store()
        inst = cls._instance = cls(rank, world, local_rank, device, store)
        inst.collective = world > 1 or forced
        inst.forced = forced
        if inst.collective:
            import torch.distributed as dist

            inst._cpu_group()
            inst._init_shm()
            # weight collectives run on their own group over the live ranks: the watchdog may abort
            # it (ncclCommAbort) without touching WORLD, whose store later groups rendezvous on
            inst._pg = dist.new_group(ranks=list(range(world)))
            inst._start_watchdog()
        if store is not None and world > 1:
            inst.bus = StoreBus(store, rank, world, inst._deliver)
        return inst

    @classmethod
    def _init_mesh(cls, devs: List[torch.device], backend: Optional[str]) -> "Federation":
        from myfyp_amd.parallel.device_mesh import make_mesh

        if devs[0].type == "cuda":
            torch.cuda.set_device(devs[0])
        inst = cls._instance = cls(0, 1, 0, devs[0], None)
        inst.devices = list(devs)
        physical = all(d.type == "cuda" for d in devs) and len({d.index for d in devs}) == len(devs)
        try:
            inst.mesh = make_mesh(devs, backend)
        except Exception as e:  # noqa: BLE001 — RCCL init on this host failed
            if backend is not None or (physical and not Settings.MESH_HOST_FALLBACK):
                # an explicitly requested backend, or distinct physical GPUs, must not be swapped
                # silently for host copies (a "mesh" number that is not RCCL)
                raise
            # opt-in (MESH_HOST_FALLBACK): the job still runs on every device, with the host
            # mesh's device-to-device copies in place of RCCL; reported as ``mesh.kind`` = "host"
            from myfyp_amd.parallel.device_mesh import HostMesh

            logger.warning("rank0", f"RCCL device mesh over {[str(d) for d in devs]} failed ({e}); using the host mesh")
            print(f"[federation] RCCL device mesh failed ({e}); falling back to the host mesh", file=sys.stderr, flush=True)
            inst.mesh = HostMesh(devs)
        inst.mesh_members = list(range(len(devs)))
        from myfyp_amd.parallel.mesh_guard import MeshGuard

        inst.mesh_guard = MeshGuard(inst)
        logger.info("rank0", f"device mesh over {[str(d) for d in devs]} ({inst.mesh.kind})")
        return inst

    @property
    def mesh_size(self) -> int:
        return len(self.mesh_members) if self.mesh is not None else 1

    def placement(self) -> Optional[Tuple[str, int]]:
        """Next peer's (device, mesh rank), round-robin over the mesh (None outside a mesh)."""
        if self.mesh is None:
            return None
        with self._lock:
            r = self.mesh_members[self._placed % len(self.mesh_members)]
            self._placed += 1
        return str(self.devices[r]), r

    def mesh_position(self, mesh_rank: int) -> int:
        """Index of an original mesh rank among the ranks still in the mesh."""
        return self.mesh_members.index(mesh_rank)

    def mesh_scratch(self, mesh_rank: int, numel: int, tag: str = "") -> torch.Tensor:
        """fp32 scratch on a mesh rank's device (a rank without live peers still joins a collective)."""
        key = (mesh_rank, numel, tag)
        t = self._mesh_scratch.get(key)
        if t is None:
            t = self._mesh_scratch[key] = torch.zeros(numel, dtype=torch.float32, device=self.devices[mesh_rank])
        return t

    def mesh_track(self, kind: str, retry: Optional[Callable[[], None]] = None, streams=None) -> None:
        """Register the mesh collective just enqueued with the mesh guard (deadline, async-error
        poll, retry from retained inputs: ``parallel/mesh_guard.py``). ``streams`` (one per
        member): where the collective ran, if not on the members' current streams."""
        g = self.mesh_guard
        if g is not None:
            g.track(kind, retry, streams)

    def mesh_confirm(self) -> bool:
        """Confirm the pending mesh collectives (recovering from a failed one); True if a
        recovery ran."""
        g = self.mesh_guard
        return g.confirm() if g is not None and self.mesh is not None else False

    def mesh_drop_ranks(self, ranks: List[int]) -> None:
        """Mesh ranks whose device stopped responding: their peers leave the experiment (they
        are unregistered now, so the current aggregation runs over the others, and stopped in the
        background: a stop may block on the lost device)."""
        lost = []
        with self._lock:
            for a in list(self.local_order):
                node = self.local_nodes.get(a)
                if node is not None and getattr(node.learner, "mesh_rank", 0) in ranks:
                    lost.append(node)
        for node in lost:
            logger.warning("rank0", f"peer {node.addr} sits on a lost device: it leaves the experiment")
            self.unregister_local(node.addr)
            threading.Thread(target=node.stop, name=f"stop-{node.addr}", daemon=True).start()

    def mesh_leave(self, mesh_rank: int) -> None:
        """A mesh rank's last peer stopped: rebuild the mesh over the other ranks; it joins no
        further collective. The mesh is healthy, so the pending collectives are confirmed and
        every member device is drained first (a collective or apply kernel of the previous round
        may still be queued: ADVICE r5), then the communicators are destroyed, not aborted, and
        a fresh init-all runs over the others."""
        if self.mesh is None or mesh_rank not in self.mesh_members or len(self.mesh_members) == 1:
            return
        self.mesh_confirm()
        if mesh_rank not in self.mesh_members or len(self.mesh_members) == 1:
            return
        t0 = time.perf_counter()
        self._mesh_rebuild([r for r in self.mesh_members if r != mesh_rank])
        self.record("mesh_shrink", time.perf_counter() - t0)
        logger.warning("rank0", f"mesh rank {mesh_rank} ({self.devices[mesh_rank]}) has no live peer: mesh rebuilt over {self.mesh_members}")

    def _mesh_rebuild(self, ranks: List[int]) -> None:
        """Rebuild the healthy mesh over the mesh ranks ``ranks``: pending collectives confirmed,
        every member device drained, communicators destroyed, init-all over ``ranks``."""
        self.mesh_confirm()
        keep = [i for i, r in enumerate(self.mesh_members) if r in ranks]
        for r in self.mesh_members:
            d = self.devices[r]
            if d.type == "cuda":
                torch.cuda.synchronize(d)
        self.mesh.rebuild(keep)
        self.mesh_members = [self.mesh_members[i] for i in keep]

    def mesh_ranks_alive(self) -> List[int]:
        """Mesh ranks that still host a live local peer."""
        alive = set()
        for a in self.local_order:
            node = self.local_nodes.get(a)
            if node is None:
                continue
            r = getattr(node.learner, "mesh_rank", None)
            alive.add(0 if r is None else r)
        return [r for r in self.mesh_members if r in alive]

    def mesh_sync(self) -> None:
        """Drop mesh ranks without live peers (called between rounds)."""
        if self.mesh is None:
            return
        alive = self.mesh_ranks_alive()
        for r in [r for r in self.mesh_members if r not in alive]:
            if len(self.mesh_members) > 1 and alive:
                self.mesh_leave(r)

    @classmethod
    def get(cls) -> "Federation":
        if cls._instance is None:
            return cls.init()
        return cls._instance

    def _init_shm(self) -> None:
        """All ranks on one host (the single-node MI355X case) → control-plane gathers go through a
        shared-memory segment (``csrc/host/shm_collective.cpp``) instead of gloo TCP."""
        if not Settings.SHM_CONTROL_PLANE or self.store is None:
            return
        import socket

        from myfyp_amd.parallel.shm_collective import ShmCollective

        try:
            with open("/proc/sys/kernel/random/boot_id") as f:
                host = socket.gethostname() + "/" + f.read().strip()
        except OSError:
            host = socket.gethostname()
        self.store.set(f"fedhost/{self.rank}", host)
        if any(self.store.get(f"fedhost/{r}").decode() != host for r in range(self.world)):
            return
        self.shm = ShmCollective.create(self.store, self.rank, self.world, timeout=float(Settings.COLLECTIVE_TIMEOUT))
        if self.shm is not None:
            self.shm.heartbeat()

            def beat() -> None:
                while not self._hb_stop.wait(0.1):
                    shm = self.shm
                    if shm is None:
                        return
                    shm.heartbeat()

            self._hb_thread = threading.Thread(target=beat, name=f"fed-heartbeat-{self.rank}", daemon=True)
            self._hb_thread.start()

    def _stop_watchdog(self) -> None:
        self._wd_stop.set()
        t, self._wd_thread = self._wd_thread, None
        if t is not None and t is not threading.current_thread():
            t.join(timeout=5.0)

    def _stop_heartbeat(self) -> None:
        self._hb_stop.set()
        t, self._hb_thread = self._hb_thread, None
        if t is not None and t is not threading.current_thread():
            t.join(timeout=5.0)

    def shutdown(self) -> None:
        """Leave the job, wait until every rank has left (the rendezvous store lives in rank 0's
        process), stop the control bus and tear down the process groups (call once, at exit).
        Departed ranks take the same path, so a job with a dead peer still ends cleanly."""
        synced = False
        if self.central is not None:
            self.central.stop()  # last flush to rank 0 while every rank is still here
            self.central = None
        try:
            self.confirm_collectives()  # the last round's device collective (nothing to re-run after it)
        except Exception as e:
            logger.warning(f"rank{self.rank}", f"last collective unconfirmed at shutdown: {e}")
        self._pending.clear()
        self._stop_watchdog()
        if self.bus is not None:
            self.bus.stop()
            self.bus = None
        # Process groups go first and the shm "all gone" wait last: rank 0's process hosts the
        # rendezvous store, so it must not exit while another rank is still tearing down its groups
        # (a store that vanished under a peer's destroy_process_group aborted that peer at exit).
        if self.collective:
            import torch.distributed as dist

            if dist.is_initialized():
                if self.shm is None and not self.departed and self.members == list(range(self.world)) and not self._aborted:
                    dist.barrier(group=self._pg)
                dist.destroy_process_group()
        if self.mesh is not None:
            try:
                self.mesh_confirm()  # the last round's mesh collectives (a failure is recovered)
                self.mesh.check()
            except Exception as e:
                logger.warning(f"rank{self.rank}", f"mesh collectives unconfirmed at shutdown: {e}")
            if self.mesh_guard is not None:
                self.mesh_guard.stop()
            for r in self.mesh_members:
                d = self.devices[r]
                if d.type == "cuda":
                    torch.cuda.synchronize(d)
            self.mesh.close()
            self.mesh = None
        if self.shm is not None:
            self.shm.leave()
            synced = self.shm.wait_all_gone(float(Settings.COLLECTIVE_TIMEOUT), float(Settings.FAILURE_TIMEOUT))
            if not synced:
                logger.warning(f"rank{self.rank}", "not every rank left within COLLECTIVE_TIMEOUT")
            self._stop_heartbeat()  # joined before the unmap: a beat in flight wrote into freed pages (SIGSEGV at exit)
            self.shm.close()
            self.shm = None
        Federation._instance = None

    @classmethod
    def reset(cls) -> None:
        inst = cls._instance
        if inst is not None and inst.central is not None:
            inst.central.stop()
            inst.central = None
        if inst is not None and inst.bus is not None:
            inst.bus.stop()
        if inst is not None:
            inst._stop_watchdog()
            inst._stop_heartbeat()
        if inst is not None and inst.shm is not None:
            inst.shm.close()
            inst.shm = None
        if inst is not None and inst.mesh_guard is not None:
            inst.mesh_guard.stop()
        if inst is not None and inst.mesh is not None:
            try:
                for d in inst.devices:
                    if d.type == "cuda":
                        torch.cuda.synchronize(d)
                inst.mesh.close()
            except Exception as e:  # best effort (a test tearing down after a failure)
                logger.debug("rank0", f"mesh close: {e}")
            inst.mesh = None
        cls._instance = None

    def register_local(self, node) -> None:
        with self._lock:
            self.local_nodes[node.addr] = node
            if node.addr not in self.local_order:
                self.local_order.append(node.addr)

    def finalize(self, connect: bool = True) -> List[str]:
        """Exchange the peer lists of all ranks and connect every local node to every peer."""
        local = list(self.local_order)
        if self.world > 1:
            import json

            self.store.set(f"members/{self.rank}", json.dumps(local))
            for r in range(self.world):
                self.store.wait([f"members/{r}"])
                for addr in json.loads(self.store.get(f"members/{r}")):
                    self.peers[addr] = r
        else:
            for addr in local:
                self.peers[addr] = 0
        if connect:
            for addr in local:
                node = self.local_nodes[addr]
                for other in self.peers:
                    if other != addr:
                        node.communication_protocol.connect(other)
        if self.world > 1 and float(Settings.CENTRAL_LOG_PERIOD) > 0 and self.central is None:
            from myfyp_amd.management.logger import logger
            from myfyp_amd.management.logger.central import CentralLogRelay

            self.central = CentralLogRelay(self, logger)
        self.finalized.set()
        return self.all_peers()

    def all_peers(self) -> List[str]:
        return sorted(self.peers, key=lambda a: (self.peers[a], a))

    def is_local(self, addr: str) -> bool:
        return addr in self.local_nodes

    def remote_stub(self, addr: str) -> Optional[RemotePeer]:
        r = self.peers.get(addr)
        if r is None or r == self.rank or self.bus is None:
            return None
        return RemotePeer(self, r, addr)

    def _deliver(self, dest: str, kind: str, msg: dict) -> None:
        from myfyp_amd.communication.protocols.memory.memory_communication_protocol import ServerRegistry
        from myfyp_amd.management.logger.central import RELAY_ADDR, RELAY_KIND

        if dest == RELAY_ADDR and kind == RELAY_KIND:  # live metrics of another rank (rank 0 only)
            if self.central is not None:
                self.central.ingest(msg)
            else:
                from myfyp_amd.management.logger import logger

                logger.ingest_records([tuple(r) for r in msg.get("records") or []])
            return

        server = ServerRegistry.get(dest)
        if server is None:
            return
        if kind == "weights":
            server.handle_weights(msg)
        else:
            server.handle_message(msg)

    # ------------------------------------------------------------------ collectives (gang leaders only)
    def live_local(self) -> List[str]:
        return [a for a in self.local_order if a in self.local_nodes and self.local_nodes[a].state.round is not None]

    def round_driver(self):
        """Lock-step round driver of the co-located peers (stages/collective/driver.py)."""
        with self._lock:
            if self._round_driver is None:
                from myfyp_amd.stages.collective.driver import RoundDriver

                self._round_driver = RoundDriver(self)
            return self._round_driver

    def gang_run(self, member: str, payload: Any, fn: Callable[[Dict[str, Any]], Any], timeout: Optional[float] = None) -> Any:
        def members() -> List[str]:
            return [a for a in self.local_order if a in self.local_nodes]

        return self.gang.run(member, members, payload, fn, Settings.AGGREGATION_TIMEOUT if timeout is None else timeout)

    def unregister_local(self, addr: str, mid_experiment: bool = False) -> None:
        """A co-located peer stopped (or crashed): drop it from every future gang. If it was the
        last live local peer and an experiment was running, this rank departs the federation."""
        with self._lock:
            self.local_nodes.pop(addr, None)
            last = not self.local_nodes
        self.gang.poke()
        if last and mid_experiment:
            self.depart()

    # ------------------------------------------------------------------ membership
    def depart(self) -> None:
        """This rank leaves the running experiment: it joins no further collective, and the other
        ranks stop waiting for it at their next gather (shared-memory membership protocol)."""
        if self.departed or not self.collective:
            return
        # under the section lock: a weights section that already gathered the membership (and so
        # counts on this rank) must see the departure only at its exit (reading
        # _frozen unlocked let a rank leave between the gather and the freeze)
        with self._section_lock:
            self.departed = True
            if self._frozen is not None:
                # inside a weights section this rank already agreed to take part: it completes the
                # section's collectives and leaves at its exit (the others would wait for it otherwise)
                self._depart_deferred = True
            elif self.shm is not None:
                self._leave_clean()
        logger.warning(f"rank{self.rank}", "last local peer stopped mid-experiment: rank departs the federation")

    def _leave_clean(self) -> None:
        """Leave the shm membership on purpose. The deferred device collectives this rank joined
        are completed locally first, so the others, when they confirm them, see a rank that left
        after finishing them (``left_clean``) rather than one that failed inside them: no recovery,
        and the confirmed round result keeps the leaver's share."""
        deadline = time.perf_counter() + float(Settings.COLLECTIVE_TIMEOUT)
        all_done = True
        for works, _, _, _ in self._pending:
            for w in works:
                if w is None:
                    continue
                while True:
                    try:
                        if w.is_completed():
                            break
                    except Exception:  # a failed collective is not a completed one
                        all_done = False
                        break
                    if time.perf_counter() >= deadline:
                        all_done = False
                        break
                    time.sleep(0.0005)
        self._pending.clear()
        # kLeft ("left clean") only when every collective this rank joined was seen to complete;
        # otherwise leave as an eviction, so the survivors recover instead of trusting its share
        # 
        if not all_done:
            logger.warning(f"rank{self.rank}", "leaving with unconfirmed collectives: the others will treat this rank as failed")
        self.shm.leave(clean=all_done)

    def _apply_members(self, ranks: List[int], force: bool = False) -> None:
        """Every survivor calls this with the same participant set at the same gather (``force``:
        rebuild the groups even when nobody left, after a failed collective aborted them)."""
        if ranks == self.members and not force:
            return
        import torch.distributed as dist

        gone = [r for r in self.members if r not in ranks]
        if gone:
            logger.warning(f"rank{self.rank}", f"ranks {gone} left the federation; continuing over ranks {ranks}")
        with self._lock:
            self.members = list(ranks)
            self.peers = {a: r for a, r in self.peers.items() if r in ranks}
        # process groups over the survivors; group-local rendezvous (the departed ranks take no part)
        old = (self._pg, self._cpu_pg)
        self._pg = dist.new_group(ranks=ranks, use_local_synchronization=True)
        self._cpu_pg = self._pg if dist.get_backend() == "gloo" else dist.new_group(ranks=ranks, backend="gloo", use_local_synchronization=True)
        # the replaced groups include a rank that is gone: abort them (local, never blocks on the
        # dead rank the way a destroy would) so their communicators and buffers are released
        for g in {id(x): x for x in old if x is not None and x is not dist.group.WORLD}.values():
            self._release_group(g)
        self.record("membership_change", float(len(gone)))

    def sync_members(self) -> List[int]:
        """Liveness agreement right before a weight collective (a peer may have died since the
        round's vote gather): every survivor leaves with the same member list and process group."""
        if self.collective and not self.departed and self.shm is not None:
            t0 = time.perf_counter()
            ranks, _ = self.shm.allgather_members(None, float(Settings.FAILURE_TIMEOUT))
            self.record("cp_sync_members", time.perf_counter() - t0)
            if ranks != self.members and self._pending:
                # a collective left unconfirmed by the confirmation lag still runs on the old group:
                # confirm it first (recovering if it failed), as when it was confirmed before this
                # gather, then agree again — every survivor saw the same change and takes this path
                self.confirm_collectives()
                ranks, _ = self.shm.allgather_members(None, float(Settings.FAILURE_TIMEOUT))
            self._apply_members(ranks)
        return self.members

    def all_gather_object(self, obj: Any) -> List[Any]:
        """Control-plane gather (votes, wire models) over a CPU (gloo) group: an object gather on the
        RCCL group would pickle through device memory and synchronise the host with every queued
        kernel, stalling the asynchronous round pipeline."""
        if not self.collective or self._is_departed():
            return [obj]
        if self.shm is not None:
            t0 = time.perf_counter()
            ranks, got = self.shm.allgather_members(obj, float(Settings.FAILURE_TIMEOUT))
            self.record("cp_gather", time.perf_counter() - t0)
            self._apply_members(ranks)
            if got is not None:
                return [got[r] for r in ranks]
            # some rank's payload exceeded the shared slot: every member takes the gloo path together
        import torch.distributed as dist

        out: List[Any] = [None] * len(self.members)
        dist.all_gather_object(out, obj, group=self._cpu_group())
        return out

    def gather_logs(self) -> None:
        """Collective (every rank calls it): merge every rank's metric stores into every rank's
        logger, so ``logger.get_global_logs()`` shows all peers of the job (the reference's
        multi-process runs centralise logs in one Ray actor, ``ray_logger.py:32-250``)."""
        if not self.collective:
            return
        from myfyp_amd.management.logger import logger

        mine = (self.rank, logger.get_global_logs(), logger.get_local_logs())
        for rank, g, loc in self.all_gather_object(mine):
            if rank != self.rank:
                logger.merge_logs(g, loc)

    def _cpu_group(self):
        if self._cpu_pg is None:
            import torch.distributed as dist

            self._cpu_pg = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
        return self._cpu_pg

    def all_reduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place all-reduce over RCCL among the live ranks (bucketed for large buffers). Guarded:
        returns only once every member completed it; raises :class:`MembershipChanged` (groups
        rebuilt, ``t`` restored to its input) when a member died inside it."""
        if not self.collective or self._is_departed():
            return t
        import torch.distributed as dist

        rop = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
        flat = t.view(-1)
        keep = flat.clone() if self._guarded() else None
        self._pre_collective("all_reduce")
        bucket = max(1, Settings.BUCKET_BYTES // flat.element_size())
        t0 = time.perf_counter()
        works = [dist.all_reduce(flat[i : i + bucket], op=rop, group=self._pg, async_op=True) for i in range(0, flat.numel(), bucket)]
        try:
            self.await_works(works, "all_reduce")
        except MembershipChanged:
            if keep is not None:
                flat.copy_(keep)
            raise
        self.comm.host("all_reduce", flat.numel() * flat.element_size(), time.perf_counter() - t0)
        return t

    def all_reduce_async(self, t: torch.Tensor):
        """Start a sum all-reduce of ``t`` (one bucket) over the live ranks on the communicator's
        stream, ordered after the work already queued on the CURRENT stream. Returns the work
        handle (``wait()`` makes the current stream wait on it), or None when there is nobody to
        reduce with."""
        if self.solo:
            return None
        import torch.distributed as dist

        self._pre_collective("all_reduce_async")
        self.comm.host("all_reduce_async", t.numel() * t.element_size(), 0.0)
        return dist.all_reduce(t, group=self._pg, async_op=True)

    def all_gather_into_tensor_(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """Guarded ``all_gather_into_tensor`` over the live ranks (same contract as ``all_reduce_``)."""
        import torch.distributed as dist

        t0 = time.perf_counter()
        self._pre_collective("all_gather")
        w = dist.all_gather_into_tensor(out, inp, group=self._pg, async_op=True)
        self.await_works([w], "all_gather")
        self.comm.host("all_gather", out.numel() * out.element_size(), time.perf_counter() - t0)
        return out

    def batch_p2p_(self, ops_: list) -> None:
        """Guarded grouped point-to-point sends/receives (topology mixing)."""
        import torch.distributed as dist

        t0 = time.perf_counter()
        # gloo's send/recv works only complete inside wait() (a dead peer's closed socket raises there)
        self.await_works(dist.batch_isend_irecv(ops_), "p2p", poll=dist.get_backend(self._pg) != "gloo")
        self.comm.host("p2p", 0, time.perf_counter() - t0)

    def broadcast_(self, t: torch.Tensor, src_rank: int) -> torch.Tensor:
        if not self.collective or self._is_departed():
            return t
        import torch.distributed as dist

        t0 = time.perf_counter()
        self._pre_collective("broadcast")
        w = dist.broadcast(t, src=src_rank, group=self._pg, async_op=True)
        self.await_works([w], "broadcast")
        self.comm.host("broadcast", t.numel() * t.element_size(), time.perf_counter() - t0)
        return t

    @property
    def solo(self) -> bool:
        """No other live rank to exchange weights with (a forced single-rank RCCL job is not solo:
        its collectives run through RCCL)."""
        if not self.collective or self._is_departed():
            return True
        return self.members == [self.rank] and not self.forced

    # ------------------------------------------------------------------ collective guard
    def _pre_collective(self, kind: str) -> None:
        for hook in list(self.pre_collective_hooks):
            hook(kind)

    def _is_departed(self) -> bool:
        fz = self._frozen
        return fz[0] if fz is not None else self.departed

    def _guarded(self) -> bool:
        """Failure-aware collectives (liveness polling + agreement) need the shared-memory control
        plane (single-node jobs); elsewhere collectives fall back to the RCCL/gloo timeouts."""
        return bool(Settings.COLLECTIVE_FAILOVER) and self.shm is not None

    @contextlib.contextmanager
    def weights_section(self):
        """One aggregation's weight collectives. Membership is agreed once at entry (one shm
        gather) and frozen with this rank's departure state until exit, so a rank that agreed to
        take part always completes the collectives it agreed to (a concurrent ``depart()`` takes
        effect at exit). Nested sections reuse the outer agreement."""
        with self._section_lock:
            mark("section:in")
            outer = self._frozen is not None
            if not outer and self.mesh is not None:
                # the previous round's mesh collectives are confirmed (a failed one is recovered:
                # abort, rebuild over the responsive devices, re-run from the retained partials),
                # then devices whose last peer stopped leave the mesh
                self.mesh_confirm()
                self.mesh_sync()
            if not outer:
                # a confirmation that ended in an agreement gather already agreed on the members
                # (every member took part in it): no second membership gather right after it
                if not self.confirm_collectives(force=False):
                    self.sync_members()
                self._frozen = (self.departed, list(self.members))
            try:
                yield self
            finally:
                if not outer:
                    self._frozen = None
                    if self._depart_deferred:
                        self._depart_deferred = False
                        if self.shm is not None:
                            self._leave_clean()

    def run_aggregation(self, fn: Callable[[], Any]) -> Any:
        """Run ``fn`` (an aggregation: reads the local rows, weight collectives, then writes) in a
        weights section; when a member died inside one of its collectives the groups are rebuilt
        and ``fn`` is re-run over the survivors (its inputs are intact: nothing is written before
        the last collective returned on every member)."""
        for attempt in range(self.world + 1):
            try:
                with self.weights_section():
                    return fn()
            except MembershipChanged as e:
                logger.warning(f"rank{self.rank}", f"re-running the aggregation over ranks {self.members} ({e})")
        raise RuntimeError("aggregation did not complete after repeated membership changes")

    def _members_alive(self, members: List[int]) -> List[int]:
        """Members (other than this rank) that are unresponsive right now, or already evicted by
        another rank's gather. The evicted ones matter to a rank still waiting inside the
        collective: the faster survivors evicted the dead rank and moved on to the agreement, so
        neither its heartbeat nor the others' progress would ever end this rank's wait (the 8-rank
        rehearsal hung this way about once in ten runs). A member that left on purpose completed
        the collectives it had joined and does not count."""
        if self.shm is None:
            return []
        bad = set(self.shm.unresponsive(float(Settings.FAILURE_TIMEOUT)))
        alive = set(self.shm.alive())
        if len(alive) < self.world:
            clean = set(self.shm.left_clean())
            bad |= {r for r in members if r not in alive and r not in clean}
        return [r for r in sorted(bad) if r in members and r != self.rank]

    def await_works(self, works: list, what: str, poll: bool = True) -> None:
        """Wait for collective works while watching the members' liveness; then agree with the
        other members that every one of them completed (one shm gather). On a failure anywhere:
        abort the group, re-agree membership over the survivors and raise MembershipChanged."""
        works = [w for w in works if w is not None]
        if not self._guarded():
            for w in works:
                w.wait()
            return
        members = list(self._frozen[1]) if self._frozen is not None else list(self.members)
        group = self._pg
        ok = True
        self._inflight = (group, members)
        try:
            spin = 0
            for w in works:
                while True:
                    try:
                        if not poll or w.is_completed():
                            w.wait()  # surfaces an error; makes the current stream wait (nccl)
                            break
                    except Exception as e:  # connection closed by a dead peer (gloo), aborted comm (nccl)
                        logger.warning(f"rank{self.rank}", f"{what} failed: {str(e)[:160]}")
                        ok = False
                        break
                    if id(group) in self._aborted or self._members_alive(members):
                        ok = False
                        break
                    spin += 1
                    time.sleep(0 if spin < 200 else 0.0005)
                if not ok:
                    break
        finally:
            self._inflight = None
        self._agree(ok, group, what)

    def _agree(self, ok: bool, group, what: str) -> None:
        """Every member reports whether its collective completed; unless all did and nobody left,
        everyone aborts the group, rebuilds over the survivors and re-runs."""
        t0 = time.perf_counter()
        ranks, got = self.shm.allgather_members(bool(ok), float(Settings.FAILURE_TIMEOUT))
        self.record("cp_agree", time.perf_counter() - t0)
        frozen = self._frozen[1] if self._frozen is not None else self.members
        # a member missing from the gather is fine only if it left on purpose: it completed the
        # collectives it had joined before leaving (depart / _leave_clean); an evicted one did not
        missing = [r for r in frozen if r not in ranks]
        clean = set(self.shm.left_clean()) if missing else set()
        all_ok = ok and got is not None and all(bool(got[r]) for r in ranks) and set(ranks) <= set(frozen) and all(r in clean for r in missing)
        if all_ok:
            if missing:
                logger.info(f"rank{self.rank}", f"{what}: ranks {missing} left after completing it")
                # the gather agreed the new member set (every member took part): adopt it, also
                # for the frozen view of a deferred confirmation. Collectives still pending on the
                # old group are confirmed first: rebuilding aborts the old group, which would fail
                # them and trigger the recovery a clean leave is meant to avoid
                if self._pending and what != "deferred all_reduce":
                    self._confirm_pending()
                self._apply_members(ranks)
                if self._frozen is not None:
                    self._frozen = (self._frozen[0], list(self.members))
            return
        self.recoveries += 1
        self.record("collective_recovery", 1.0)
        self._release_group(group)
        self._apply_members(ranks, force=True)
        if self._frozen is not None:
            self._frozen = (self._frozen[0], list(self.members))
        raise MembershipChanged(f"{what}: members {list(frozen)} -> {ranks}")

    def _release_group(self, g) -> None:
        """Abort a replaced/failed device group (ncclCommAbort: local, never blocks on the dead
        rank the way a destroy would, ends kernels still waiting on it, frees the communicator)."""
        import torch.distributed as dist

        if g is None or g is dist.group.WORLD or id(g) in self._aborted:
            return
        self._aborted.add(id(g))
        try:
            # gloo: a waiter on a dead peer already fails on its closed socket, and aborting a gloo
            # group tears its worker threads down under the waiter (std::terminate): just drop it
            if dist.get_backend(g) != "gloo":
                dist.distributed_c10d._abort_process_group(g)
        except Exception as e:  # best effort: the group is never used again
            logger.debug(f"rank{self.rank}", f"group abort: {e}")

    def _start_watchdog(self) -> None:
        """Background watchdog: while a weight collective is in flight, a member that becomes
        unresponsive gets the group aborted, so device kernels stuck on the dead peer end (the
        host-side waits notice the abort and recover)."""
        if not self._guarded() or self._wd_thread is not None:
            return

        def run() -> None:
            while not self._wd_stop.wait(0.02):
                inf = self._inflight
                pend = self._pending
                cands = [inf] if inf is not None else []
                cands += [(g, m) for _, m, _, g in pend]
                for g, members in cands:
                    if g is not None and id(g) not in self._aborted and self._members_alive(members):
                        logger.warning(f"rank{self.rank}", f"watchdog: member(s) {self._members_alive(members)} unresponsive inside a collective; aborting the group")
                        self._release_group(g)

        self._wd_thread = threading.Thread(target=run, name=f"fed-watchdog-{self.rank}", daemon=True)
        self._wd_thread.start()

    def defer_confirm(self, works: list, retry: Callable[[], None]) -> None:
        """Register an asynchronous weight collective (device pipeline: apply kernels already
        queued behind it) whose outcome is confirmed before the next aggregation or round —
        ``retry`` re-runs it over the survivors from retained inputs."""
        if not self._guarded():
            return
        members = list(self._frozen[1]) if self._frozen is not None else list(self.members)
        self._pending.append((works, members, retry, self._pg))

    def confirm_collectives(self, force: bool = True) -> bool:
        """Confirm the deferred device collectives (every member completed them); on a failure
        the groups are rebuilt and the retained-input retry runs (synchronously confirmed).

        ``force`` False (the weights-section entry, ``Settings.CONFIRM_LAG``): a newest collective
        not yet complete on the device waits one more section; the others are confirmed.

        Called at the next weights-section entry: the round's all-reduce r is confirmed while the
        next local epoch r+1 — already queued behind it — runs, so confirming never idles the GPU
        (confirming at the top of the next round instead cost 20 % of the MLP round rate:
        ``profiles/r3a_rccl_forced``). The price is paid only on a failure: epoch r+1 then started
        from rows the failed all-reduce left behind; the retry writes the survivors' average of
        round r over them, so round r+1's local progress is discarded and every survivor continues
        from the same, correct, round-r model."""
        if not self._pending:
            return False
        # lag (not forced): the newest collective, while still queued behind the running epoch, is
        # left for the next section (or shutdown), so the round driver keeps launching ahead
        # instead of waiting for the GPU to reach it; older ones are confirmed now. On a failure the
        # oldest failed entry's retry re-runs the exchange from the partial sums retained last (the
        # newest round's) over the survivors, and every newer entry is dropped with the group
        keep_last = (not force and self._confirm_lag and not self._pending_complete(self._pending[-1]))
        if keep_last and len(self._pending) == 1:
            return False
        t0 = time.perf_counter()
        try:
            self._confirm_pending(keep_last)
        finally:
            self.record("cp_confirm", time.perf_counter() - t0)
        return self._guarded() and not self._is_departed()

    @property
    def _confirm_lag(self) -> bool:
        return bool(Settings.CONFIRM_LAG) and os.environ.get("MYFYP_CONFIRM_LAG", "1") != "0"

    @staticmethod
    def _pending_complete(entry) -> bool:
        """Non-blocking: every work of a deferred entry has completed on the device (a work that
        raises counts as complete: confirming it surfaces the failure)."""
        for w in entry[0]:
            if w is None:
                continue
            try:
                if not w.is_completed():
                    return False
            except Exception:  # noqa: BLE001 — an aborted communicator: confirm now
                return True
        return True

    def _confirm_pending(self, keep_last: bool = False) -> None:
        while len(self._pending) > (1 if keep_last else 0):
            works, members, retry, _ = self._pending.pop(0)
            with self._section_lock:
                saved = self._frozen
                self._frozen = (False, members)
                try:
                    self.await_works(works, "deferred all_reduce")
                except MembershipChanged as e:
                    logger.warning(f"rank{self.rank}", f"re-running a deferred collective over ranks {self.members} ({e})")
                    self._frozen = None
                    self._pending.clear()
                    try:
                        self.run_aggregation(retry)
                    finally:
                        self._frozen = saved
                    self.confirm_collectives()
                    return
                finally:
                    # restored on every exit (a gather timeout or a failed retry included): a stale
                    # frozen state would make every later weights section look nested
                    self._frozen = saved

    @property
    def group(self):
        """Device process group over the live ranks (None = the default group)."""
        return self._pg

    def barrier(self) -> None:
        if not self.collective or self.departed:
            return
        if self.shm is not None:
            self.sync_members()
            return
        import torch.distributed as dist

        dist.barrier(group=self._pg)

    def record(self, name: str, seconds: float) -> None:
        self.stats.setdefault(name, []).append(seconds)


def mesh_devices(spec: Any) -> Optional[List[torch.device]]:
    """Device list of an in-process mesh from ``spec`` (count or list of device strings), or None
    for no mesh (``spec`` None/0/1, or an empty list). A count larger than the visible GPUs raises, unless
    ``Settings.MESH_VIRTUAL`` allows a virtual mesh (every member on cuda:0, HostMesh collectives:
    a one-GPU rehearsal of the N-device path); on a CPU host the members are ``cpu``."""
    if spec is None:
        return None
    if isinstance(spec, (list, tuple)):  # an explicit member list is always a mesh (even of one)
        return [torch.device(d) for d in spec] or None
    n = int(spec)
    if n <= 1:
        return None
    if not torch.cuda.is_available():
        return [torch.device("cpu")] * n
    have = torch.cuda.device_count()
    if n <= have:
        return [torch.device("cuda", i) for i in range(n)]
    if Settings.MESH_VIRTUAL:
        return [torch.device("cuda", 0)] * n
    raise RuntimeError(f"device mesh of {n} GPUs requested, {have} visible")


def rccl_reserved_cus() -> int:
    """CUs a concurrent RCCL collective can occupy: ``Settings.RCCL_RESERVED_CUS`` if set, else the
    RCCL channel cap in force (NCCL_MAX_NCHANNELS / NCCL_MAX_CTAS, RCCL's own knobs; RCCL launches
    one workgroup per channel), else ``Settings.RCCL_MAX_CHANNELS``."""
    if Settings.RCCL_RESERVED_CUS is not None:
        return int(Settings.RCCL_RESERVED_CUS)
    caps = [int(os.environ[k]) for k in ("NCCL_MAX_NCHANNELS", "NCCL_MAX_CTAS") if os.environ.get(k, "").isdigit()]
    return min(caps) if caps else int(Settings.RCCL_MAX_CHANNELS)


def _default_store():
    import torch.distributed as dist

    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500")) + 1
        return dist.TCPStore(addr, port, int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")) == 0)
