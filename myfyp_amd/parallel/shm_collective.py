"""Node-local control-plane collectives over shared memory (``csrc/host/shm_collective.cpp``).

The collective workflow gathers a few hundred bytes per round across ranks (train-set votes; the
reference broadcasts them as TTL-relayed ``vote_train_set`` messages,
``p2pfl/stages/base_node/vote_train_set_stage.py:101-107``). On one MI355X node every rank shares
the host, so the exchange is a shared-memory all-gather: a release store per rank and a spin on
the others — microseconds instead of the two gloo TCP collectives of ``all_gather_object``.

Payloads larger than the slot (e.g. wire-format models for non-stacked learners) make *every* rank
fall back to the gloo group in the same call, so ranks never diverge.
"""

from __future__ import annotations

import ctypes
import os
import pickle
import secrets
from typing import Any, Dict, List, Optional, Tuple

from myfyp_amd.management.logger import logger

_LIB: Optional[ctypes.CDLL] = None


def _load() -> Optional[ctypes.CDLL]:
    global _LIB
    if _LIB is not None:
        return _LIB
    from myfyp_amd.ops.build import HOST_LIB, build_host

    path = HOST_LIB
    if not os.path.exists(path):
        try:
            path = build_host()
        except Exception as e:  # no compiler: gloo path
            logger.debug("", f"shm control plane unavailable: {e}")
            return None
    lib = ctypes.CDLL(path)
    vp, i, u64, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_double
    lib.shmc_open.restype = vp
    lib.shmc_open.argtypes = [ctypes.c_char_p, i, i, u64, i, d]
    lib.shmc_wait_attached.restype = i
    lib.shmc_wait_attached.argtypes = [vp, d]
    lib.shmc_unlink.restype = i
    lib.shmc_unlink.argtypes = [ctypes.c_char_p]
    lib.shmc_slot_bytes.restype = u64
    lib.shmc_slot_bytes.argtypes = [vp]
    lib.shmc_allgather.restype = i
    lib.shmc_allgather.argtypes = [vp, ctypes.c_char_p, u64, vp, ctypes.POINTER(u64), d]
    lib.shmc_barrier.restype = i
    lib.shmc_barrier.argtypes = [vp, d]
    lib.shmc_allgather_m.restype = i
    lib.shmc_allgather_m.argtypes = [vp, ctypes.c_char_p, u64, vp, ctypes.POINTER(u64), ctypes.POINTER(u64), d, d]
    lib.shmc_leave.restype = i
    lib.shmc_leave.argtypes = [vp]
    lib.shmc_leave_ex.restype = i
    lib.shmc_leave_ex.argtypes = [vp, i]
    lib.shmc_heartbeat.restype = None
    lib.shmc_heartbeat.argtypes = [vp]
    lib.shmc_alive.restype = u64
    lib.shmc_alive.argtypes = [vp]
    lib.shmc_left_clean.restype = u64
    lib.shmc_left_clean.argtypes = [vp]
    lib.shmc_state.restype = ctypes.c_int
    lib.shmc_state.argtypes = [vp, vp]
    lib.shmc_wait_all_gone.restype = i
    lib.shmc_wait_all_gone.argtypes = [vp, d, d]
    lib.shmc_unresponsive.restype = u64
    lib.shmc_unresponsive.argtypes = [vp, d]
    lib.shmc_close.restype = None
    lib.shmc_close.argtypes = [vp]
    _LIB = lib
    return lib


class ShmCollective:
    """One shared segment per job; created by rank 0, name agreed through the rendezvous store.

    The name is unlinked as soon as every rank attached, so nothing is left in ``/dev/shm`` even if
    a rank is killed later.
    """

    def __init__(self, handle: int, rank: int, world: int, timeout: float) -> None:
        lib = _load()
        assert lib is not None
        self._lib = lib
        self._h = ctypes.c_void_p(handle)
        self.rank, self.world, self.timeout = rank, world, timeout
        self.slot = int(lib.shmc_slot_bytes(self._h))
        self._out = ctypes.create_string_buffer(self.slot * world)
        self._lens = (ctypes.c_uint64 * world)()

    @classmethod
    def create(cls, store, rank: int, world: int, slot_bytes: int = 64 << 10, timeout: float = 300.0, key: str = "shmc") -> Optional["ShmCollective"]:
        """Collective over all ranks (every rank must call it). Returns None on every rank if any
        rank could not attach (then the caller keeps the gloo path)."""
        lib = _load()
        ok_local = lib is not None
        name = b""
        handle = None
        if rank == 0:
            if ok_local:
                name = f"/myfyp_{os.getpid()}_{secrets.token_hex(6)}".encode()
                handle = lib.shmc_open(name, 0, world, slot_bytes, 1, timeout)
                ok_local = bool(handle)
            store.set(f"{key}/name", name.decode() if ok_local else "")
        else:
            name = store.get(f"{key}/name")
            ok_local = ok_local and bool(name)
            if ok_local:
                handle = lib.shmc_open(name, rank, world, slot_bytes, 0, 30.0)
                ok_local = bool(handle)
        store.set(f"{key}/ok/{rank}", "1" if ok_local else "0")
        all_ok = all(store.get(f"{key}/ok/{r}") == b"1" for r in range(world))
        if all_ok and lib.shmc_wait_attached(handle, timeout) != 0:
            all_ok = False
        if rank == 0 and name:
            lib.shmc_unlink(name)
        if not all_ok:
            if handle:
                lib.shmc_close(handle)
            return None
        return cls(handle, rank, world, timeout)

    def allgather_bytes(self, data: bytes) -> Optional[List[bytes]]:
        """All ranks' payloads, or None (on every rank) if one of them did not fit its slot."""
        rc = self._lib.shmc_allgather(self._h, data, len(data), ctypes.addressof(self._out), self._lens, self.timeout)
        if rc < 0:
            raise TimeoutError(f"shared-memory all-gather timed out after {self.timeout}s (a rank died or stalled)")
        if rc == 1:
            return None
        base = ctypes.addressof(self._out)
        return [ctypes.string_at(base + r * self.slot, int(self._lens[r])) for r in range(self.world)]

    def allgather_object(self, obj: Any) -> Optional[List[Any]]:
        parts = self.allgather_bytes(pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL))
        if parts is None:
            return None
        return [pickle.loads(p) for p in parts]  # payloads written by this job's own ranks

    # ------------------------------------------------------------------ membership (fault tolerance)
    def allgather_members(self, obj: Any, fail_s: float) -> Tuple[List[int], Optional[Dict[int, Any]]]:
        """All-gather over the ranks still in the job: (participant ranks, {rank: payload}) — the
        same participant set on every survivor. A rank whose heartbeat is older than ``fail_s`` is
        evicted. Payload dict None (on every participant) if one payload overflowed its slot."""
        mask = ctypes.c_uint64(0)
        data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        rc = self._lib.shmc_allgather_m(self._h, data, len(data), ctypes.addressof(self._out), self._lens, ctypes.byref(mask), self.timeout, fail_s)
        if rc == -3:
            raise RuntimeError("this rank left the federation (or was evicted as unresponsive)")
        if rc < 0:
            raise TimeoutError(f"shared-memory all-gather timed out after {self.timeout}s")
        ranks = [r for r in range(self.world) if mask.value >> r & 1]
        if rc == 1:
            return ranks, None
        base = ctypes.addressof(self._out)
        return ranks, {r: pickle.loads(ctypes.string_at(base + r * self.slot, int(self._lens[r]))) for r in ranks}

    def leave(self, clean: bool = True) -> bool:
        """Leave the job: later all-gathers of the other ranks no longer wait for this one.
        ``clean=False``: leave as if evicted (the others must not count on this rank having
        completed the collectives it joined)."""
        return self._lib.shmc_leave_ex(self._h, 1 if clean else 0) == 0

    def heartbeat(self) -> None:
        self._lib.shmc_heartbeat(self._h)

    def alive(self) -> List[int]:
        m = int(self._lib.shmc_alive(self._h))
        return [r for r in range(self.world) if m >> r & 1]

    def state(self) -> Tuple[int, List[str]]:
        """Diagnostics: (this rank's generation, every rank's status word; G = gone, L = left clean)."""
        buf = (ctypes.c_uint64 * (self.world + 1))()
        self._lib.shmc_state(self._h, ctypes.addressof(buf))
        out = []
        for r in range(self.world):
            s = int(buf[1 + r])
            out.append(("G" + ("L" if s >> 62 & 1 else "") + str(s & ((1 << 62) - 1))) if s >> 63 else str(s))
        return int(buf[0]), out

    def left_clean(self) -> List[int]:
        """Ranks that left on purpose (``leave``) — as opposed to evicted as unresponsive."""
        m = int(self._lib.shmc_left_clean(self._h))
        return [r for r in range(self.world) if m >> r & 1]

    def unresponsive(self, fail_s: float) -> List[int]:
        """Member ranks (other than this one) whose process is gone or whose heartbeat is older
        than ``fail_s`` — read-only; the collective watchdog's trigger."""
        m = int(self._lib.shmc_unresponsive(self._h, fail_s))
        return [r for r in range(self.world) if m >> r & 1]

    def wait_all_gone(self, timeout: float, fail_s: float = 0.0) -> bool:
        """Job end: wait until every rank left; a crashed rank (process gone, or heartbeat older
        than ``fail_s``) is evicted instead of waited for."""
        return self._lib.shmc_wait_all_gone(self._h, timeout, fail_s) == 0

    def barrier(self) -> None:
        if self._lib.shmc_barrier(self._h, self.timeout) != 0:
            raise TimeoutError(f"shared-memory barrier timed out after {self.timeout}s")

    def close(self) -> None:
        if self._h:
            self._lib.shmc_close(self._h)
            self._h = ctypes.c_void_p()
