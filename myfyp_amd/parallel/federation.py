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
  eviction (``heartbeater.py:94-103``) for the RCCL weights plane.
"""

from __future__ import annotations

import datetime
import os
import sys
import pickle
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from myfyp_amd.management.logger import logger
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

    def host(self, kind: str, nbytes: int, seconds: float) -> None:
        with self._lock:
            self._add(kind, nbytes, seconds * 1e6)

    def device(self, kind: str, nbytes: int, ev0, ev1) -> None:
        with self._lock:
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

    # ------------------------------------------------------------------ lifecycle
    @classmethod
    def init(cls, backend: Optional[str] = None) -> "Federation":
        """Initialise from ``torchrun`` env vars (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*)."""
        if cls._instance is not None:
            return cls._instance
        if Settings.GIL_SWITCH_INTERVAL:
            sys.setswitchinterval(float(Settings.GIL_SWITCH_INTERVAL))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if torch.cuda.is_available():
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
            device = torch.device("cuda", torch.cuda.current_device())
        else:
            device = torch.device("cpu")
        store = None
        if world > 1:
            import torch.distributed as dist

            if not dist.is_initialized():
                # MYFYP_DIST_BACKEND=gloo rehearses a multi-rank job on ONE GPU (RCCL refuses two
                # ranks on one device); production multi-GPU jobs use RCCL ("nccl")
                be = backend or os.environ.get("MYFYP_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
                kw = {"timeout": datetime.timedelta(seconds=Settings.COLLECTIVE_TIMEOUT)}
                if be == "nccl":
                    kw["device_id"] = device
                dist.init_process_group(backend=be, **kw)
            store = _default_store()
        cls._instance = cls(rank, world, local_rank, device, store)
        if world > 1:
            cls._instance._cpu_group()
            cls._instance._init_shm()
        if store is not None:
            cls._instance.bus = StoreBus(store, rank, world, cls._instance._deliver)
        return cls._instance

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
        if self.shm is not None:
            self.shm.leave()
            synced = self.shm.wait_all_gone(float(Settings.COLLECTIVE_TIMEOUT))
            self._stop_heartbeat()  # joined before the unmap: a beat in flight wrote into freed pages (SIGSEGV at exit)
            self.shm.close()
            self.shm = None
        if self.bus is not None:
            self.bus.stop()
            self.bus = None
        if self.world > 1:
            import torch.distributed as dist

            if dist.is_initialized():
                if not synced and not self.departed:
                    dist.barrier(group=self._pg)
                dist.destroy_process_group()
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
            inst._stop_heartbeat()
        if inst is not None and inst.shm is not None:
            inst.shm.close()
            inst.shm = None
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
        if self.departed or self.world == 1:
            return
        self.departed = True
        if self.shm is not None:
            self.shm.leave()
        logger.warning(f"rank{self.rank}", "last local peer stopped mid-experiment: rank departs the federation")

    def _apply_members(self, ranks: List[int]) -> None:
        """Every survivor calls this with the same participant set at the same gather."""
        if ranks == self.members:
            return
        import torch.distributed as dist

        gone = [r for r in self.members if r not in ranks]
        logger.warning(f"rank{self.rank}", f"ranks {gone} left the federation; continuing over ranks {ranks}")
        with self._lock:
            self.members = list(ranks)
            self.peers = {a: r for a, r in self.peers.items() if r in ranks}
        # process groups over the survivors; group-local rendezvous (the departed ranks take no part)
        self._pg = dist.new_group(ranks=ranks, use_local_synchronization=True)
        self._cpu_pg = self._pg if dist.get_backend() == "gloo" else dist.new_group(ranks=ranks, backend="gloo", use_local_synchronization=True)
        self.record("membership_change", float(len(gone)))

    def sync_members(self) -> List[int]:
        """Liveness agreement right before a weight collective (a peer may have died since the
        round's vote gather): every survivor leaves with the same member list and process group."""
        if self.world > 1 and not self.departed and self.shm is not None:
            ranks, _ = self.shm.allgather_members(None, float(Settings.FAILURE_TIMEOUT))
            self._apply_members(ranks)
        return self.members

    def all_gather_object(self, obj: Any) -> List[Any]:
        """Control-plane gather (votes, wire models) over a CPU (gloo) group: an object gather on the
        RCCL group would pickle through device memory and synchronise the host with every queued
        kernel, stalling the asynchronous round pipeline."""
        if self.world == 1 or self.departed:
            return [obj]
        if self.shm is not None:
            ranks, got = self.shm.allgather_members(obj, float(Settings.FAILURE_TIMEOUT))
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
        if self.world == 1:
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
        """In-place all-reduce over RCCL among the live ranks (bucketed for large buffers)."""
        if self.world == 1 or self.departed:
            return t
        import torch.distributed as dist

        rop = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
        flat = t.view(-1)
        bucket = max(1, Settings.BUCKET_BYTES // flat.element_size())
        t0 = time.perf_counter()
        if flat.numel() <= bucket:
            dist.all_reduce(flat, op=rop, group=self._pg)
        else:
            works = [dist.all_reduce(flat[i : i + bucket], op=rop, group=self._pg, async_op=True) for i in range(0, flat.numel(), bucket)]
            for w in works:
                w.wait()
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

        self.comm.host("all_reduce_async", t.numel() * t.element_size(), 0.0)
        return dist.all_reduce(t, group=self._pg, async_op=True)

    def broadcast_(self, t: torch.Tensor, src_rank: int) -> torch.Tensor:
        if self.world == 1 or self.departed:
            return t
        import torch.distributed as dist

        t0 = time.perf_counter()
        dist.broadcast(t, src=src_rank, group=self._pg)
        self.comm.host("broadcast", t.numel() * t.element_size(), time.perf_counter() - t0)
        return t

    @property
    def solo(self) -> bool:
        """No other live rank to exchange weights with."""
        return self.world == 1 or self.departed or self.members == [self.rank]

    @property
    def group(self):
        """Device process group over the live ranks (None = the default group)."""
        return self._pg

    def barrier(self) -> None:
        if self.world == 1 or self.departed:
            return
        if self.shm is not None:
            self.sync_members()
            return
        import torch.distributed as dist

        dist.barrier(group=self._pg)

    def record(self, name: str, seconds: float) -> None:
        self.stats.setdefault(name, []).append(seconds)


def _default_store():
    import torch.distributed as dist

    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500")) + 1
        return dist.TCPStore(addr, port, int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")) == 0)
