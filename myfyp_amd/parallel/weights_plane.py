"""Round-level weight collectives executed by a local gang leader (see ``federation.py``).

All functions receive ``arrived: {addr: payload}`` for the co-located peers that reached the gang
and run identically on every rank (same call order ⇒ matching RCCL collectives).
"""

from __future__ import annotations

import os
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from myfyp_amd import ops
from myfyp_amd.management.tracing import mark, traced
from myfyp_amd.parallel.federation import Federation


# ---------------------------------------------------------------------------------------------
# learner state access
# ---------------------------------------------------------------------------------------------
def state_tensors(learner) -> List[torch.Tensor]:
    """Device tensors that define a peer's model: flat trainable vector + floating buffers."""
    out = [learner.flat_params()]
    module = learner.model.get_model()
    for b in module.buffers():
        if b.is_floating_point():
            out.append(b)
    return out


def on_device(dev: torch.device):
    """Make ``dev`` the thread's current GPU (no-op for CPU members)."""
    import contextlib

    return torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext()


def mesh_rank_of(learner) -> int:
    r = getattr(learner, "mesh_rank", None)
    return 0 if r is None else int(r)


def _by_mesh_rank(fed: Federation, addrs, learners) -> Dict[int, List[Tuple[str, Any]]]:
    out: Dict[int, List[Tuple[str, Any]]] = {r: [] for r in fed.mesh_members}
    for a, lr in zip(addrs, learners):
        r = mesh_rank_of(lr)
        if r not in out:
            raise RuntimeError(f"peer {a} sits on mesh rank {r}, which left the mesh")
        out[r].append((a, lr))
    return out


def _stacked_group(learners) -> Optional[Any]:
    """Return the shared MLPGroup when every learner is a row of one stacked buffer."""
    groups = {id(getattr(lr, "_engine", None) and lr._engine.group) for lr in learners}
    if len(groups) != 1 or getattr(learners[0], "_engine", None) is None:
        return None
    return learners[0]._engine.group


# ---------------------------------------------------------------------------------------------
# initial model (reference: init_model gossip, start_learning_stage.py:82-112)
# ---------------------------------------------------------------------------------------------
def sync_initial_model(fed: Federation, arrived: Dict[str, Any], initiator: str) -> None:
    """Every peer adopts the initiator's weights: local copy + one RCCL broadcast per dtype (the
    state tensors are packed into one flat buffer each, so ResNet-18's ~100 tensors cost one
    guarded broadcast and one agreement gather, not one per tensor: ADVICE r3)."""
    learners = {a: fed.local_nodes[a].learner for a in arrived if a in fed.local_nodes}
    if fed.mesh is not None:
        _mesh_initial_model(fed, learners, initiator)
        return

    def run() -> None:
        # the initiator's rank, or (if it died) the lowest survivor: every survivor agrees on it
        src_rank = fed.peers.get(initiator, min(fed.members))
        if src_rank not in fed.members:
            src_rank = min(fed.members)
        ref_addr = initiator if initiator in learners else next(iter(learners))
        src = state_tensors(learners[ref_addr])
        groups: Dict[Any, List[int]] = {}
        for i, t in enumerate(src):
            groups.setdefault((t.dtype, t.device), []).append(i)
        bufs: List[Any] = [None] * len(src)
        for idx in groups.values():
            flat = torch.cat([src[i].detach().reshape(-1) for i in idx])
            fed.broadcast_(flat, src_rank)
            for i, part in zip(idx, torch.split(flat, [src[i].numel() for i in idx])):
                bufs[i] = part.view_as(src[i])
        with torch.no_grad():
            for a, lr in learners.items():
                for dst, s in zip(state_tensors(lr), bufs):
                    dst.copy_(s)

    fed.run_aggregation(run)


def _mesh_initial_model(fed: Federation, learners: Dict[str, Any], initiator: str) -> None:
    """Device mesh: pack the initiator's state tensors per dtype on its device, ONE RCCL broadcast
    per dtype from its mesh rank, unpack into every peer of every device."""
    ref_addr = initiator if initiator in learners else next(iter(learners))
    root_r = mesh_rank_of(learners[ref_addr])
    root = fed.mesh_position(root_r)
    src = state_tensors(learners[ref_addr])
    groups: Dict[Any, List[int]] = {}
    for i, t in enumerate(src):
        groups.setdefault(t.dtype, []).append(i)
    per_rank: Dict[int, List[Any]] = {r: [None] * len(src) for r in fed.mesh_members}
    for dt, idx in groups.items():
        numel = sum(src[i].numel() for i in idx)
        flats = []
        for r in fed.mesh_members:
            dev = fed.devices[r]
            if r == root_r:
                flats.append(torch.cat([src[i].detach().reshape(-1) for i in idx]).to(dev))
            else:
                flats.append(torch.empty(numel, dtype=dt, device=dev))
        fed.mesh.broadcast_(flats, root)
        fed.mesh_track("broadcast")
        for r, flat in zip(fed.mesh_members, flats):
            for i, part in zip(idx, torch.split(flat, [src[i].numel() for i in idx])):
                per_rank[r][i] = part.view_as(src[i])
    with torch.no_grad():
        for a, lr in learners.items():
            r = mesh_rank_of(lr)
            with on_device(fed.devices[r]):
                for dst, s_ in zip(state_tensors(lr), per_rank[r]):
                    dst.copy_(s_)


# ---------------------------------------------------------------------------------------------
# votes
# ---------------------------------------------------------------------------------------------
def gather_votes(fed: Federation, arrived: Dict[str, Dict[str, int]]) -> Dict[str, Dict[str, int]]:
    allv: Dict[str, Dict[str, int]] = {}
    for part in fed.all_gather_object(dict(arrived)):
        allv.update(part)
    return allv


# ---------------------------------------------------------------------------------------------
# aggregation
# ---------------------------------------------------------------------------------------------
_COMM_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


def comm_stream(dev: torch.device) -> "torch.cuda.Stream":
    """The side HIP stream that carries the weight collectives of ``dev`` (one per device)."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _COMM_STREAMS.get(idx)
    if st is None:
        st = _COMM_STREAMS[idx] = torch.cuda.Stream(device=idx)
    return st


def bucket_ranges(n: int, bucket_bytes: int) -> List[Tuple[int, int]]:
    """[b0, b1) ranges over n floats; every b0 is a multiple of 4 (float4 kernels stay aligned)."""
    step = max(4, (bucket_bytes // 4) // 4 * 4)
    return [(b0, min(n, b0 + step)) for b0 in range(0, n, step)] or [(0, 0)]


class _Delayed:
    """Delayed-averaging state of one stacked group or of the generic per-learner path."""

    def __init__(self) -> None:
        self.snap: Optional[torch.Tensor] = None  # round-r local rows (stacked: [capacity, n])
        self.snaps: Dict[str, torch.Tensor] = {}  # generic path: addr -> packed row
        self.buf: Optional[torch.Tensor] = None  # [wsum, pad x3 | Σ w x_r] (stacked) / [Σ w x_r | Σ w] (generic)
        self.done = None  # event on the side stream: the round-r all-reduce has landed in buf
        self.pending = False


def _delayed_state(fed: Federation, key) -> _Delayed:
    table = fed.__dict__.setdefault("_delayed", {})
    st = table.get(key)
    if st is None:
        st = table[key] = _Delayed()
    return st


def _stacked_mean_cuda(fed: Federation, group, w: np.ndarray, mask: np.ndarray, final: bool) -> None:
    """FedAvg of a stacked ``[capacity, S]`` group on the GPU, host never waits.

    * one rank: one ``k_fedavg_local`` launch (weighted mean written into every masked row);
    * several ranks, ``OVERLAP_COLLECTIVES``: per bucket a reduce launch (which also writes the
      failover's retained copy) and an async all-reduce on RCCL's stream, ordered after that launch,
      then per bucket wait + apply launch — bucket k's all-reduce overlaps bucket k+1's reduce and
      bucket k-1's apply. These run on the compute stream itself: the next epoch needs the average,
      and a side stream only put two more cross-stream hops on the round's critical path
      (``profiles/r6k_forced_trace``);
    * ``DELAYED_AVERAGING`` (opt-in, not on the last round): land the previous round's average as
      ``x += avg - snap`` and take the new snapshot (one launch), then reduce + all-reduce the
      snapshot on the side stream while the next round trains from the local weights.
    """
    from myfyp_amd.settings import Settings

    fast = ops.fast_lib()
    n, P, S = group.numel, group.capacity, group.S
    dev = group.params.device
    cur = torch.cuda.current_stream(dev)
    wp, mp = w.ctypes.data, mask.ctypes.data
    base = group.params.data_ptr()
    delayed = bool(Settings.DELAYED_AVERAGING)
    st = _delayed_state(fed, id(group)) if (delayed or getattr(fed, "_delayed", {}).get(id(group))) else None
    landed = False
    if st is not None and st.pending:  # land round r-1's average (and re-snapshot) in one launch
        cur.wait_event(st.done)
        ops.check(fast.myfyp_fedavg_delayed_land(base, st.snap.data_ptr(), n, st.buf.data_ptr() + 16, st.buf.data_ptr(), P, n, S, mp, cur.cuda_stream),
                  "fedavg_delayed_land")
        st.pending, landed = False, True
    if delayed and not final:
        if st.snap is None or tuple(st.snap.shape) != (P, n):
            # zeros: rows of unused capacity slots are read (with weight 0) by the reduce
            st.snap = torch.zeros(P, n, dtype=torch.float32, device=dev)
            st.buf = torch.zeros(n + 4, dtype=torch.float32, device=dev)
            landed = False
        if not landed:  # first delayed round: snapshot only
            ops.check(fast.myfyp_fedavg_delayed_land(base, st.snap.data_ptr(), n, None, None, P, n, S, mp, cur.cuda_stream), "fedavg_snapshot")
        snap_ptr, sbuf = st.snap.data_ptr(), st.buf
        works = _bucketed_reduce(fed, fast, comm_stream(dev), cur, snap_ptr, n, n, P, wp, sbuf, apply=None)
        st.done = torch.cuda.Event()
        st.done.record(comm_stream(dev))
        st.pending = True

        def retry() -> None:  # the snapshot rows are intact: reduce them again over the survivors
            c = torch.cuda.current_stream(dev)
            # the failed bucketed reduce / all-reduce wrote sbuf on the comm stream
            c.wait_stream(comm_stream(dev))
            ops.check(fast.myfyp_fedavg_bucket_reduce(sbuf.data_ptr() + 16, sbuf.data_ptr(), snap_ptr, P, n, n, w.ctypes.data, c.cuda_stream),
                      "fedavg_bucket_reduce")
            fed.all_reduce_(sbuf)
            st.done = torch.cuda.Event()
            st.done.record(c)

        fed.defer_confirm(works, retry)
        return
    if fed.solo:  # nothing to all-reduce: weighted mean and write-back in one launch
        mark("agg:launch")
        ops.check(fast.myfyp_fedavg_stacked_local(base, P, n, S, wp, mp, cur.cuda_stream), "fedavg_local")
        mark("agg:launched")
        return
    if not Settings.OVERLAP_COLLECTIVES:
        buf = group.fedavg_buffer()
        ops.check(fast.myfyp_fedavg_stacked_reduce(buf.data_ptr(), base, P, n, S, wp, cur.cuda_stream), "fedavg_reduce")
        fed.all_reduce_(buf)
        ops.check(fast.myfyp_fedavg_stacked_apply(base, buf.data_ptr(), P, n, S, mp, cur.cuda_stream), "fedavg_apply")
        return
    buf = getattr(group, "_wp_bucket_buf", None)
    if buf is None or buf.numel() != n + 4:
        buf = group._wp_bucket_buf = torch.zeros(n + 4, dtype=torch.float32, device=dev)
    keep = None
    if fed._guarded():  # retained local partial sums: a failed all-reduce is re-run from them
        keep = getattr(group, "_wp_keep_buf", None)
        if keep is None or keep.numel() != n + 4:
            keep = group._wp_keep_buf = torch.zeros(n + 4, dtype=torch.float32, device=dev)
    # on the compute stream: the next epoch needs the average anyway, and the buckets still pipeline
    # (bucket k's all-reduce runs on RCCL's stream while bucket k + 1 reduces); a side stream only
    # added two cross-stream hops to the round's critical path (profiles/r6k_forced_trace)
    side = os.environ.get("MYFYP_FEDAVG_SIDE", "0") == "1"  # A/B: the side-stream pipeline of round 5
    works = _bucketed_reduce(fed, fast, comm_stream(dev) if side else cur, cur, base, S, n, P, wp, buf, apply=(base, S, mp), keep=keep)
    if keep is not None:

        def retry() -> None:  # survivors: all-reduce the retained local partials, apply again
            c = torch.cuda.current_stream(dev)
            c.wait_stream(comm_stream(dev))
            buf.copy_(keep)
            fed.all_reduce_(buf)
            ops.check(fast.myfyp_fedavg_bucket_apply(base, buf.data_ptr() + 16, buf.data_ptr(), P, n, S, mask.ctypes.data, c.cuda_stream),
                      "fedavg_bucket_apply")

        fed.defer_confirm(works, retry)


def _bucketed_reduce(fed: Federation, fast, cs, cur, src: int, ld: int, n: int, P: int, wp: int, buf: torch.Tensor, apply, keep=None) -> list:
    """Side-stream pipeline over ``bucket_ranges``: reduce launch + async all-reduce per bucket,
    then (``apply`` = (dst, ld, mask)) per bucket wait + apply launch. ``buf`` = [wsum, pad x3 | data];
    bucket 0's all-reduce carries the weight sum, so apply k needs only buckets 0 and k. ``keep``
    (failover) receives a copy of each bucket's local partial sum before its all-reduce. Returns
    the all-reduce works (confirmed later by the collective guard)."""
    from myfyp_amd.settings import Settings

    same = cs.cuda_stream == cur.cuda_stream  # critical path: everything on the compute stream
    if not same:
        cs.wait_stream(cur)  # the rows are final on the compute stream
    bp = buf.data_ptr()
    kp = keep.data_ptr() if keep is not None else None
    ranges = bucket_ranges(n, Settings.BUCKET_BYTES)
    works = []
    timed = fed.comm.timed("fedavg_pipeline")
    ev0, ev1 = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if timed else (None, None)
    if timed:
        ev0.record(cs)
    with torch.cuda.stream(cs):
        for k, (b0, b1) in enumerate(ranges):
            if kp is None:
                ops.check(fast.myfyp_fedavg_bucket_reduce(bp + 4 * (4 + b0), bp if k == 0 else None, src + 4 * b0, P, b1 - b0, ld, wp, cs.cuda_stream),
                          "fedavg_bucket_reduce")
            else:  # the retained copy from the same pass (no device copy behind it)
                ops.check(fast.myfyp_fedavg_bucket_reduce2(bp + 4 * (4 + b0), bp if k == 0 else None, kp + 4 * (4 + b0), kp if k == 0 else None,
                                                           src + 4 * b0, P, b1 - b0, ld, wp, cs.cuda_stream), "fedavg_bucket_reduce2")
            lo = 0 if k == 0 else 4 + b0
            works.append(fed.all_reduce_async(buf[lo : 4 + b1]))
        for k, (b0, b1) in enumerate(ranges):
            if works[k] is not None:
                works[k].wait()
            if apply is not None:
                dst, dld, mp = apply
                ops.check(fast.myfyp_fedavg_bucket_apply(dst + 4 * b0, bp + 4 * (4 + b0), bp, P, b1 - b0, dld, mp, cs.cuda_stream), "fedavg_bucket_apply")
    if timed:
        ev1.record(cs)
    fed.comm.device("fedavg_pipeline", 4 * (n + 1), ev0, ev1)  # resolved lazily by the node monitor (sampled timing)
    if not same:
        buf.record_stream(cs)
        if keep is not None:
            keep.record_stream(cs)
        if apply is not None:
            cur.wait_stream(cs)  # stream-level: the next kernel on the compute stream sees the average
    return works


@traced("aggregate_mean")
def aggregate_mean(fed: Federation, arrived: Dict[str, Tuple[float, Any]], final: bool = True) -> Tuple[float, List[str]]:
    """Sample-weighted mean of the trainers' models (weight 0 for non-trainers), result into every
    local peer. Stacked groups on the GPU: see ``_stacked_mean_cuda`` (side-stream bucketed
    pipeline, optional delayed averaging). ``final`` marks the experiment's last round (delayed
    averaging flushes and aggregates exactly there)."""
    from myfyp_amd.settings import Settings

    t0 = time.perf_counter()

    def run() -> Tuple[float, List[str]]:
        mark("agg:run")
        addrs = [a for a in arrived if a in fed.local_nodes]  # a peer may die after arriving
        learners = [fed.local_nodes[a].learner for a in addrs]
        weights = [float(arrived[a][0]) for a in addrs]
        contributors = [a for a, w in zip(addrs, weights) if w > 0]
        if fed.mesh is not None:
            mut = _MeshMutation(fed, addrs)
            out = _mesh_mean(fed, addrs, learners, weights, final)
            if mut.before:
                mut.apply()
            return out, contributors
        group = _stacked_group(learners)
        dev = learners[0].flat_params().device
        if group is not None and dev.type == "cuda":
            w = np.zeros(group.capacity, dtype=np.float32)
            mask = np.zeros(group.capacity, dtype=np.float32)
            for lr, wt in zip(learners, weights):
                w[lr._engine.slot] = wt
                mask[lr._engine.slot] = 1.0
            _stacked_mean_cuda(fed, group, w, mask, final)
            total_w = float(sum(weights))  # local share; the global Σw stays on the device
        elif group is not None:
            wm = torch.zeros(2, group.capacity, dtype=torch.float32)
            for lr, wt in zip(learners, weights):
                wm[0, lr._engine.slot] = wt
                wm[1, lr._engine.slot] = 1.0
            n = group.numel
            buf = torch.empty(n + 1, dtype=torch.float32, device=dev)
            ops.stacked_weighted_sum(group.params[:, :n], wm[0], buf[:n], 1.0)
            buf[n:].fill_(float(sum(weights)))
            fed.all_reduce_(buf)
            total = buf[n:].clone()
            buf[:n].div_(total.clamp_min(1e-12))
            ops.broadcast_rows(buf[:n], group.params[:, :n], wm[1])
            total_w = total
        else:
            total_w = _generic_mean(fed, addrs, learners, weights, final, bool(Settings.DELAYED_AVERAGING))
        return total_w, contributors

    # the side-stream pipeline's all-reduces stay unconfirmed until the next weights section (or
    # shutdown): by then the next local epoch is already queued behind them, so the host's wait for
    # them never leaves the GPU idle (see Federation.confirm_collectives)
    total_w, contributors = fed.run_aggregation(run)
    fed.record("aggregate", time.perf_counter() - t0)
    return total_w, contributors


def _mesh_mean(fed: Federation, addrs, learners, weights, final: bool = True) -> float:
    """FedAvg over a device mesh. Stacked engine groups (one per mesh rank): ONE native call.
    With ``OVERLAP_COLLECTIVES`` (default) it is the bucketed exchange on each device's comm
    stream (``rmesh_fedavg_bucketed``: reduce, per-bucket grouped all-reduce, the compute stream
    waiting per bucket for its apply; ``DELAYED_AVERAGING`` runs it beside the next local epoch and
    lands it a round later — see :func:`_mesh_mean_bucketed`); otherwise per device reduce launch,
    one grouped RCCL all-reduce and per device apply launch on the compute streams
    (``rmesh_fedavg``). Other learners: per device partial sums, one mesh all-reduce, unpack.

    The all-reduce is out of place, so every device keeps its local partial sum [Σ w x | Σ w]. The
    mesh guard (``parallel/mesh_guard.py``) confirms the collective at the next weights section;
    if it failed (asynchronous RCCL error, or a device that never completed it within
    ``COLLECTIVE_TIMEOUT``), the mesh is rebuilt over the responsive devices and ``retry`` re-runs
    the all-reduce of the retained partial sums over them and re-applies: the survivors' average
    of the round, i.e. the models that arrived (``aggregator.py:177-208``)."""
    wt_of = dict(zip(addrs, weights))
    ranks = _by_mesh_rank(fed, addrs, learners)
    groups = {r: {id(lr._engine.group): lr._engine.group for _, lr in v if getattr(lr, "_engine", None) is not None} for r, v in ranks.items()}
    stacked = all(len(g) == 1 and len(groups[r]) == 1 for r, g in groups.items() if ranks[r]) and all(
        getattr(lr, "_engine", None) is not None for v in ranks.values() for _, lr in v)
    numels = {next(iter(g.values())).numel for g in groups.values() if g}
    from myfyp_amd.settings import Settings

    if stacked and len(numels) == 1 and (Settings.OVERLAP_COLLECTIVES or Settings.DELAYED_AVERAGING or getattr(fed, "_mesh_delayed", None)):
        return _mesh_mean_bucketed(fed, ranks, groups, numels.pop(), wt_of, float(sum(weights)), bool(Settings.DELAYED_AVERAGING) and not final)
    if stacked and len(numels) == 1 and all(next(iter(g.values())).params.is_cuda for g in groups.values() if g):
        n = numels.pop()
        per: Dict[int, tuple] = {}  # mesh rank -> (params, partial, result, P, ld, w, mask)
        for r in fed.mesh_members:
            if ranks[r]:
                g = next(iter(groups[r].values()))
                wr = np.zeros(g.capacity, dtype=np.float32)
                mr = np.zeros(g.capacity, dtype=np.float32)
                for a, lr in ranks[r]:
                    wr[lr._engine.slot] = wt_of[a]
                    mr[lr._engine.slot] = 1.0
                with on_device(g.device):
                    out = getattr(g, "_mesh_out", None)
                    if out is None or out.numel() != n + 1:
                        out = g._mesh_out = torch.empty(n + 1, dtype=torch.float32, device=g.device)
                    per[r] = (g.params, g.fedavg_buffer(), out, g.capacity, g.S, wr, mr)
            else:  # no live peer on this device (yet in the mesh): contributes zeros
                scratch = fed.mesh_scratch(r, n + 1)
                per[r] = (scratch, scratch, fed.mesh_scratch(r, n + 1, "out"), 0, n, np.zeros(0, np.float32), np.zeros(0, np.float32))

        def cols(k: int, rs) -> list:
            return [per[r][k] for r in rs]

        rs = list(fed.mesh_members)
        fed.mesh.fedavg_stacked(cols(0, rs), cols(1, rs), cols(3, rs), n, cols(4, rs), np.concatenate(cols(5, rs)),
                                np.concatenate(cols(6, rs)), outs=cols(2, rs))

        def retry() -> None:  # over the current (rebuilt) mesh: the survivors' retained partials
            live = [r for r in fed.mesh_members if r in per]
            fed.mesh.fedavg_retry(cols(0, live), cols(1, live), cols(2, live), cols(3, live), n, cols(4, live), np.concatenate(cols(6, live)))

        fed.mesh_track("fedavg", retry)
        return float(sum(weights))
    ref = _pack(learners[0])
    n = ref.numel()
    accs: Dict[int, torch.Tensor] = {}
    for r in fed.mesh_members:
        dev = fed.devices[r]
        with on_device(dev):
            acc = torch.zeros(n + 1, dtype=torch.float32, device=dev)
            for a, lr in ranks[r]:
                if wt_of[a] > 0:
                    acc[:n].add_(_pack(lr), alpha=wt_of[a])
            acc[n] = float(sum(wt_of[a] for a, _ in ranks[r]))
        accs[r] = acc  # retained partial sum (the all-reduce below works on a copy)

    def reduce_unpack() -> None:
        live = [r for r in fed.mesh_members if r in accs]
        outs = []
        for r in live:
            with on_device(fed.devices[r]):
                outs.append(accs[r].clone())
        fed.mesh.all_reduce_(outs)
        for r, out in zip(live, outs):
            with on_device(fed.devices[r]):
                avg = out[:n] / out[n].clamp_min(1e-12)
                for a, lr in ranks[r]:
                    if a in fed.local_nodes:
                        _unpack_into(lr, avg)

    reduce_unpack()
    fed.mesh_track("fedavg", reduce_unpack)
    return float(sum(weights))


def _mesh_buf(g, name: str, numel: int) -> torch.Tensor:
    """A zero-initialised fp32 buffer cached on an engine group (its device)."""
    t = getattr(g, name, None)
    if t is None or t.numel() != numel:
        with on_device(g.params.device):
            t = torch.zeros(numel, dtype=torch.float32, device=g.params.device)
        setattr(g, name, t)
    return t


def _mesh_mean_bucketed(fed: Federation, ranks, groups, n: int, wt_of, total_w: float, delayed: bool) -> float:
    """Bucketed, overlapped mesh FedAvg of stacked engine groups.

    ``rmesh_fedavg_bucketed``: per device the weighted partial sums [Σw, pad | Σ w x] go to a
    retained buffer (``keep``) on the device's comm stream, each bucket of ``BUCKET_BYTES`` is
    all-reduced (grouped over the mesh) as soon as it is reduced, and the compute stream waits per
    bucket for its apply — bucket k's apply overlaps bucket k + 1's all-reduce, and the next local
    epoch is queued behind the applies without the host waiting.

    Delayed averaging (``DELAYED_AVERAGING``, not on the last round; the ranks path's semantics,
    ``_stacked_mean_cuda``): round r - 1's exchanged average is landed as x += avg - snap together
    with the new snapshot (``rmesh_delayed_land``, one launch per device), then the snapshot rows
    are exchanged on the comm streams with no apply and nothing waiting: the whole exchange runs
    beside round r + 1's local epoch. The mesh guard watches the comm streams then.

    Failure: the guard's ``retry`` re-runs the exchange from the retained ``keep`` buffers over the
    rebuilt mesh (``rmesh_fedavg_bucketed_retry``) and re-applies — the survivors' average."""
    from myfyp_amd.settings import Settings

    bucket = max(4, int(Settings.BUCKET_BYTES) // 4)
    per: Dict[int, tuple] = {}  # mesh rank -> (params, keep, out, P, ld, w, mask, snap)
    for r in fed.mesh_members:
        if ranks[r]:
            g = next(iter(groups[r].values()))
            wr = np.zeros(g.capacity, dtype=np.float32)
            mr = np.zeros(g.capacity, dtype=np.float32)
            for a, lr in ranks[r]:
                wr[lr._engine.slot] = wt_of[a]
                mr[lr._engine.slot] = 1.0
            snap = _mesh_buf(g, "_mesh_snap", g.capacity * n) if (delayed or getattr(fed, "_mesh_delayed", None)) else None
            per[r] = (g.params, _mesh_buf(g, "_mesh_keep4", n + 4), _mesh_buf(g, "_mesh_out4", n + 4), g.capacity, g.S, wr, mr, snap)
        else:  # no live peer on this device (yet in the mesh): contributes zeros
            scratch = fed.mesh_scratch(r, n + 4, "keep4")
            per[r] = (scratch, scratch, fed.mesh_scratch(r, n + 4, "out4"), 0, n, np.zeros(0, np.float32), np.zeros(0, np.float32), scratch)

    def cols(k: int, rs) -> list:
        return [per[r][k] for r in rs]

    rs = list(fed.mesh_members)
    comm = [comm_stream(fed.devices[r]) if fed.devices[r].type == "cuda" else None for r in rs]
    mask = np.concatenate(cols(6, rs))
    if getattr(fed, "_mesh_delayed", None) is not None:  # land round r - 1's exchanged average
        fed.mesh.delayed_land(cols(0, rs), cols(7, rs), cols(2, rs), cols(3, rs), n, cols(4, rs), n, mask, True)
        fed._mesh_delayed = None
        landed = True
    else:
        landed = False
    if delayed:
        if not landed:  # first delayed round: snapshot only
            fed.mesh.delayed_land(cols(0, rs), cols(7, rs), cols(2, rs), cols(3, rs), n, cols(4, rs), n, mask, False)
        fed.mesh.fedavg_bucketed(cols(7, rs), cols(1, rs), cols(2, rs), cols(3, rs), n, [n] * len(rs), np.concatenate(cols(5, rs)), mask, comm, bucket,
                                 apply=False)
        fed._mesh_delayed = True

        def retry_delayed() -> None:  # survivors: the retained partial sums again, landed next round
            live = [r for r in fed.mesh_members if r in per]
            fed.mesh.fedavg_bucketed_retry(cols(7, live), cols(1, live), cols(2, live), cols(3, live), n, [n] * len(live), np.concatenate(cols(6, live)),
                                           apply=False)

        fed.mesh_track("fedavg (delayed)", retry_delayed, streams=comm)
        return total_w
    fed.mesh.fedavg_bucketed(cols(0, rs), cols(1, rs), cols(2, rs), cols(3, rs), n, cols(4, rs), np.concatenate(cols(5, rs)), mask, comm, bucket, apply=True)

    def retry() -> None:  # over the current (rebuilt) mesh: the survivors' retained partials
        live = [r for r in fed.mesh_members if r in per]
        fed.mesh.fedavg_bucketed_retry(cols(0, live), cols(1, live), cols(2, live), cols(3, live), n, cols(4, live), np.concatenate(cols(6, live)))

    fed.mesh_track("fedavg", retry)
    return total_w


def _generic_mean(fed: Federation, addrs, learners, weights, final: bool, delayed: bool) -> float:
    """Per-learner path (CPU, or models outside a stacked engine group); same delayed-averaging
    semantics as the stacked kernels, in torch ops."""
    st = _delayed_state(fed, "generic") if (delayed or getattr(fed, "_delayed", {}).get("generic")) else None
    if st is not None and st.pending:  # land: x += avg_{r-1} - snap_{r-1}
        avg = st.buf[:-1] / st.buf[-1].clamp_min(1e-12)
        for a, lr in zip(addrs, learners):
            if a in st.snaps:
                _unpack_into(lr, _pack(lr) + (avg - st.snaps[a]))
        st.pending = False
    rows = [_pack(lr) for lr in learners]
    n = rows[0].numel()
    acc = torch.zeros(n + 1, dtype=torch.float32, device=rows[0].device)
    for r, wt in zip(rows, weights):
        if wt > 0:
            acc[:n].add_(r, alpha=wt)
    acc[n] = sum(weights)
    fed.all_reduce_(acc)
    total_w = float(acc[n])
    if delayed and not final:  # keep the local weights; the average lands next round
        st.snaps = dict(zip(addrs, rows))
        st.buf = acc
        st.pending = True
        return total_w
    avg = acc[:n] / max(total_w, 1e-12)
    for lr in learners:
        _unpack_into(lr, avg)
    return total_w


class _MeshMutation:
    """Mutation-testing knob of the mesh aggregations (``MYFYP_DEBUG_MESH_SCALE``, default 1; never
    set in normal runs): every peer's aggregation update is scaled, x <- x_before + s·(x_agg -
    x_before), so the mesh result is off by (s - 1) of its update while the non-mesh path the GPU
    tests compare against is not. Used once to show that the mesh aggregator tests catch a 5 %
    update error (``profiles/r6_mutation``)."""

    def __init__(self, fed: Federation, addrs) -> None:
        import os

        v = os.environ.get("MYFYP_DEBUG_MESH_SCALE")
        self.scale = float(v) if v else 1.0
        self.before = {}
        if self.scale != 1.0:
            for a in addrs:
                if a in fed.local_nodes:
                    lr = fed.local_nodes[a].learner
                    self.before[a] = (lr, _pack(lr).clone())

    def apply(self) -> None:
        for lr, x0 in self.before.values():
            _unpack_into(lr, x0 + self.scale * (_pack(lr) - x0))


def _pack(learner) -> torch.Tensor:
    return torch.cat([t.detach().reshape(-1).float() for t in state_tensors(learner)])


def _unpack_into(learner, flat: torch.Tensor) -> None:
    off = 0
    with torch.no_grad():
        for t in state_tensors(learner):
            t.copy_(flat[off : off + t.numel()].view_as(t).to(t.dtype))
            off += t.numel()


@traced("aggregate_neighbors")
def aggregate_neighbors(fed: Federation, arrived: Dict[str, Any], aggregator) -> List[str]:
    """Topology mixing ``x_i ← Σ_j W_ij x_j`` (see ``NeighborAvg``): co-located rows are combined
    with the ``weighted_average`` kernel, rows of neighbours on other ranks arrive through one
    grouped batch of point-to-point sends/receives (RCCL over xGMI; gloo on CPU). Every rank calls
    this with the same peer list, so the P2P pattern matches by construction."""
    t0 = time.perf_counter()
    return fed.run_aggregation(lambda: _neighbors(fed, arrived, aggregator, t0))


def _neighbors(fed: Federation, arrived: Dict[str, Any], aggregator, t0: float) -> List[str]:
    peers = fed.all_peers()
    index = {a: i for i, a in enumerate(peers)}
    w = aggregator.mixing_matrix(len(peers))
    local = [a for a in peers if a in arrived and a in fed.local_nodes]
    if not local:
        fed.record("aggregate", time.perf_counter() - t0)
        return []
    learners = [fed.local_nodes[a].learner for a in local]
    if fed.mesh is not None and fed.mesh_size > 1:
        _mesh_neighbors(fed, peers, index, w, local, learners)
        fed.record("aggregate", time.perf_counter() - t0)
        return local
    group = _stacked_group(learners)
    if fed.solo and group is not None and group.params.is_cuda and group.capacity <= 16 and group.S % 4 == 0:
        # every neighbour is a row of the same stacked engine buffer: the whole mixing step is one
        # in-place kernel (row p <- Σ_q M[p, q] row q); no per-peer pack / average / unpack launches
        mix = np.zeros((group.capacity, group.capacity), dtype=np.float32)
        local_set = set(local)
        for a, lr in zip(local, learners):
            i = index[a]
            nz = [j for j in np.nonzero(w[i])[0] if peers[j] in local_set]  # one rank: the sources are the local arrivals
            ws = np.array([w[i, j] for j in nz], dtype=np.float64)
            ws = ws / ws.sum()
            for j, x in zip(nz, ws):
                mix[lr._engine.slot, fed.local_nodes[peers[j]].learner._engine.slot] += x
        stream = torch.cuda.current_stream(group.params.device).cuda_stream
        ops.check(ops.fast_lib().myfyp_neighbor_mix_stacked(group.params.data_ptr(), group.capacity, group.numel, group.S, mix.ctypes.data, stream),
                  "neighbor_mix")
        fed.record("aggregate", time.perf_counter() - t0)
        return local
    rows = {a: _pack(fed.local_nodes[a].learner) for a in local}
    ref = rows[local[0]]
    # point-to-point plan: every (local peer, remote rank) edge sends once; every remote neighbour is received once
    sends, recvs = {}, {}
    for a in local:
        i = index[a]
        for j in np.nonzero(w[i])[0]:
            b = peers[j]
            rb = fed.peers[b]
            if j == i or rb == fed.rank:
                continue
            sends[(a, rb)] = rows[a]
            if b not in recvs:
                recvs[b] = torch.empty_like(ref)
    if sends or recvs:
        import torch.distributed as dist

        # per rank pair, sends and receives are both ordered by the source peer's index (NCCL ignores tags)
        pg = fed.group
        ops_ = [dist.P2POp(dist.isend, t, rb, group=pg, tag=index[a]) for (a, rb), t in sorted(sends.items(), key=lambda kv: (index[kv[0][0]], kv[0][1]))]
        ops_ += [dist.P2POp(dist.irecv, t, fed.peers[b], group=pg, tag=index[b]) for b, t in sorted(recvs.items(), key=lambda kv: index[kv[0]])]
        fed.batch_p2p_(ops_)
    src = dict(rows)
    src.update(recvs)
    mixed = {}
    for a in local:
        i = index[a]
        nz = [j for j in np.nonzero(w[i])[0] if peers[j] in src]
        ws = np.array([w[i, j] for j in nz], dtype=np.float64)
        ws = ws / ws.sum()  # a dead neighbour's share folds back proportionally
        mixed[a] = ops.weighted_average([[src[peers[j]]] for j in nz], [float(x) for x in ws])[0]
    for a in local:
        _unpack_into(fed.local_nodes[a].learner, mixed[a])
    fed.record("aggregate", time.perf_counter() - t0)
    return local


def _mesh_neighbors(fed: Federation, peers, index, w, local, learners) -> None:
    """Topology mixing over a device mesh: every row a peer needs from another device arrives by
    ONE grouped RCCL send/recv exchange (``rmesh_p2p``); the mix runs on the receiving device."""
    lr_of = dict(zip(local, learners))
    rank = {a: mesh_rank_of(lr_of[a]) for a in local}
    rows = {}
    for a in local:
        with on_device(fed.devices[rank[a]]):
            rows[a] = _pack(lr_of[a])
    # (source peer, destination mesh rank) pairs, in one deterministic order for both sides
    need = sorted({(peers[j], rank[a]) for a in local for j in np.nonzero(w[index[a]])[0]
                   if peers[j] in rank and rank[peers[j]] != rank[a]}, key=lambda x: (index[x[0]], x[1]))
    got: Dict[Tuple[str, int], torch.Tensor] = {}
    ops_ = []
    for b, rd in need:
        buf = torch.empty_like(rows[b], device=fed.devices[rd])
        got[(b, rd)] = buf
        ops_.append(("send", fed.mesh_position(rank[b]), fed.mesh_position(rd), rows[b]))
        ops_.append(("recv", fed.mesh_position(rd), fed.mesh_position(rank[b]), buf))
    if ops_:
        fed.mesh.p2p_(ops_)
        fed.mesh_track("p2p")
    mixed = {}
    for a in local:
        i = index[a]
        nz = [j for j in np.nonzero(w[i])[0] if peers[j] in rank]
        ws = np.array([w[i, j] for j in nz], dtype=np.float64)
        ws = ws / ws.sum()  # a dead neighbour's share folds back proportionally
        srcs = [rows[peers[j]] if rank[peers[j]] == rank[a] else got[(peers[j], rank[a])] for j in nz]
        with on_device(fed.devices[rank[a]]):
            mixed[a] = ops.weighted_average([[t] for t in srcs], [float(x) for x in ws])[0]
    for a in local:
        with on_device(fed.devices[rank[a]]):
            _unpack_into(lr_of[a], mixed[a])


# aggregator kinds reduced on the device (no wire models, no host copies)
DEVICE_KINDS = ("mean", "neighbor", "scaffold", "median")


def _scaffold_cb(learner):
    for cb in getattr(learner, "callbacks", []):
        if cb.get_name() == "scaffold":
            return cb
    raise ValueError("SCAFFOLD aggregation needs the 'scaffold' callback on every learner")


@traced("aggregate_scaffold")
def aggregate_scaffold(fed: Federation, arrived: Dict[str, Tuple[float, Any]], aggregator) -> None:
    """SCAFFOLD server step on the device (reference math: ``p2pfl/learning/aggregators/
    scaffold.py:76-111``): x ← x_start + η_g·Σ n_i Δy_i / Σ n_i, c ← c + mean(Δc_i).

    One packed device buffer [Σ n_iΔy_i | Σ n_i | Σ Δc_i | count] reduced over the local trainers,
    ONE all-reduce over the live ranks, then every local peer's flat parameters are set to the new
    global model and its callbacks receive the new global control variate (a device tensor).
    x_start is a trainer's round-start snapshot (the callback's x0) or a non-trainer's current
    weights — identical on every rank, since every peer starts the round from the last aggregate."""
    t0 = time.perf_counter()
    fed.run_aggregation(lambda: _scaffold(fed, arrived, aggregator))
    fed.record("aggregate", time.perf_counter() - t0)


def _mesh_scaffold(fed: Federation, arrived: Dict[str, Tuple[float, Any]], aggregator) -> None:
    """SCAFFOLD server step over a device mesh: per device the packed local reduction, ONE mesh
    all-reduce, per device the apply (new model into its peers, its copy of the control variate)."""
    addrs = [a for a in arrived if a in fed.local_nodes]
    learners = [fed.local_nodes[a].learner for a in addrs]
    ranks = _by_mesh_rank(fed, addrs, learners)
    n = learners[0].flat_params().numel()
    bufs, x_starts = [], {}
    for r in fed.mesh_members:
        dev = fed.devices[r]
        dys, dcs, ws = [], [], []
        with on_device(dev):
            for a, lr in ranks[r]:
                wt = float(arrived[a][0])
                cb = _scaffold_cb(lr)
                if wt > 0 and cb.delta_y is not None:
                    dys.append(cb.delta_y)
                    dcs.append(cb.delta_c)
                    ws.append(wt)
                    x_starts.setdefault(r, cb.x0)
            buf = torch.zeros(2 * n + 2, dtype=torch.float32, device=dev)
            if dys:
                ops.scaffold_reduce(buf, dys, dcs, ws)
        bufs.append(buf)
    fed.mesh.all_reduce_(bufs)
    fed.mesh_track("scaffold all_reduce")
    cdev = fed.__dict__.setdefault("_mesh_c", {})
    for r, buf in zip(fed.mesh_members, bufs):
        if not ranks[r]:
            continue
        dev = fed.devices[r]
        with on_device(dev):
            x_start = x_starts.get(r)
            if x_start is None:  # the round-start model: every peer starts the round from it
                src = next((v for v in x_starts.values()), None)
                x_start = src.to(dev) if src is not None else ranks[r][0][1].flat_params().detach().clone()
            c_prev = cdev.get(r)
            c_init = c_prev is None or c_prev.numel() != n
            c_new = torch.empty(n, dtype=torch.float32, device=dev) if c_init else c_prev
            flats = [lr.flat_params() for _, lr in ranks[r]]
            with torch.no_grad():
                ops.scaffold_apply(flats, x_start, buf, c_new, c_init, aggregator.global_lr)
            cdev[r] = c_new
            gc = ranks[r][0][1].split_flat(c_new)
            for a, lr in ranks[r]:
                fed.local_nodes[a].aggregator._c_dev = c_new
                lr.get_model().add_info("scaffold", {"global_c": gc})
                lr.update_callbacks_with_model_info()


def _scaffold(fed: Federation, arrived: Dict[str, Tuple[float, Any]], aggregator) -> None:
    if fed.mesh is not None:  # (a one-device mesh too: its collectives still run through RCCL)
        mut = _MeshMutation(fed, list(arrived))
        _mesh_scaffold(fed, arrived, aggregator)
        if mut.before:
            mut.apply()
        return
    addrs = [a for a in arrived if a in fed.local_nodes]
    learners = {a: fed.local_nodes[a].learner for a in addrs}
    flats = [learners[a].flat_params() for a in addrs]
    n = flats[0].numel()
    dys, dcs, ws = [], [], []
    x_start = None
    for a in addrs:
        w = float(arrived[a][0])
        cb = _scaffold_cb(learners[a])
        if w > 0 and cb.delta_y is not None:
            dys.append(cb.delta_y)
            dcs.append(cb.delta_c)
            ws.append(w)
            if x_start is None:
                x_start = cb.x0
    if x_start is None:  # no local trainer: this rank's peers still hold the round-start model
        x_start = flats[0].detach().clone()
    # one reduction launch -> ONE all-reduce of [Σ n_iΔy_i | Σ n_i | Σ Δc_i | count] -> one apply
    # launch that writes the new model into every local peer and updates the control variate
    buf = torch.empty(2 * n + 2, dtype=torch.float32, device=flats[0].device)
    ops.scaffold_reduce(buf, dys, dcs, ws)
    fed.all_reduce_(buf)
    c_prev = getattr(aggregator, "_c_dev", None)
    c_init = c_prev is None or c_prev.numel() != n
    c_new = torch.empty(n, dtype=torch.float32, device=buf.device) if c_init else c_prev
    with torch.no_grad():
        ops.scaffold_apply(flats, x_start, buf, c_new, c_init, aggregator.global_lr)
    gc = learners[addrs[0]].split_flat(c_new)  # same architecture on every peer: one set of views
    for a in addrs:
        lr = learners[a]
        fed.local_nodes[a].aggregator._c_dev = c_new
        lr.get_model().add_info("scaffold", {"global_c": gc})
        lr.update_callbacks_with_model_info()


@traced("aggregate_median")
def aggregate_median(fed: Federation, arrived: Dict[str, Tuple[float, Any]]) -> None:
    """Coordinate-wise median of the trainers' models on the device (``fedmedian.py:56-62``):
    the local trainers' flat rows are packed into a [k_max, n] buffer, ONE all-gather over the live
    ranks (RCCL) collects every trainer's row, and ONE ``k_coordinate_median<K>`` launch (sorting
    network in registers, <= 16 models) writes the result into every local peer. With a single
    rank the kernel reads the live rows directly (no packing copy)."""
    t0 = time.perf_counter()
    fed.run_aggregation(lambda: _median(fed, arrived))
    fed.record("aggregate", time.perf_counter() - t0)


def _mesh_median(fed: Federation, arrived: Dict[str, Tuple[float, Any]]) -> None:
    """Coordinate median over a device mesh: every device packs its trainers' rows ([k_max, n],
    zero-padded), ONE mesh all-gather, then per device one median launch into its peers."""
    addrs = [a for a in arrived if a in fed.local_nodes]
    learners = [fed.local_nodes[a].learner for a in addrs]
    ranks = _by_mesh_rank(fed, addrs, learners)
    trainers = {r: [(a, lr) for a, lr in v if float(arrived[a][0]) > 0] for r, v in ranks.items()}
    counts = [len(trainers[r]) for r in fed.mesh_members]
    if not sum(counts):
        return
    kmax = max(counts)
    n = _pack(learners[0]).numel()
    sends, recvs = [], []
    for r in fed.mesh_members:
        dev = fed.devices[r]
        with on_device(dev):
            s_ = torch.zeros(kmax, n, dtype=torch.float32, device=dev)
            for i, (a, lr) in enumerate(trainers[r]):
                s_[i].copy_(_pack(lr))
            sends.append(s_)
            recvs.append(torch.empty(len(counts) * kmax, n, dtype=torch.float32, device=dev))
    fed.mesh.all_gather_(recvs, sends)
    fed.mesh_track("median all_gather")
    for r, recv in zip(fed.mesh_members, recvs):
        if not ranks[r]:
            continue
        with on_device(fed.devices[r]):
            rows = [recv[q * kmax + i] for q, c in enumerate(counts) for i in range(c)]
            med = torch.empty(n, dtype=torch.float32, device=recv.device)
            ops.median_into(rows, [med])
            for _, lr in ranks[r]:
                _unpack_into(lr, med)


def _median(fed: Federation, arrived: Dict[str, Tuple[float, Any]]) -> None:
    if fed.mesh is not None:  # (a one-device mesh too: its collectives still run through RCCL)
        mut = _MeshMutation(fed, list(arrived))
        _mesh_median(fed, arrived)
        if mut.before:
            mut.apply()
        return
    addrs = [a for a in arrived if a in fed.local_nodes]
    learners = {a: fed.local_nodes[a].learner for a in addrs}
    trainers = [a for a in addrs if float(arrived[a][0]) > 0]
    counts = fed.all_gather_object(len(trainers))
    kmax = max(1, max(counts))
    flat_only = all(len(state_tensors(learners[a])) == 1 for a in addrs)  # no floating buffers
    rows_of = (lambda a: learners[a].flat_params()) if flat_only else (lambda a: _pack(learners[a]))
    if fed.solo:  # every trainer is local: median straight from the live rows into every peer
        if not trainers:
            return
        if flat_only:
            ops.median_into([rows_of(a) for a in trainers], [learners[a].flat_params() for a in addrs])
        else:
            med = torch.empty_like(_pack(learners[addrs[0]]))
            ops.median_into([rows_of(a) for a in trainers], [med])
            for a in addrs:
                _unpack_into(learners[a], med)
        return
    ref = rows_of(addrs[0])
    n = ref.numel()
    send = torch.zeros(kmax, n, dtype=torch.float32, device=ref.device)
    for i, a in enumerate(trainers):
        send[i].copy_(rows_of(a))
    recv = torch.empty(len(counts) * kmax, n, dtype=torch.float32, device=ref.device)
    fed.all_gather_into_tensor_(recv, send)
    rows = [recv[r * kmax + i] for r, c in enumerate(counts) for i in range(c)]
    if not rows:
        return
    if flat_only:
        ops.median_into(rows, [learners[a].flat_params() for a in addrs])
    else:
        med = torch.empty(n, dtype=torch.float32, device=ref.device)
        ops.median_into(rows, [med])
        for a in addrs:
            _unpack_into(learners[a], med)


def aggregate_generic(fed: Federation, arrived: Dict[str, Tuple[float, Any]], aggregator) -> Any:
    """Any aggregator: all-gather the trainers' wire models and reduce identically on every rank."""
    return fed.run_aggregation(lambda: _generic(fed, arrived, aggregator))


def _generic(fed: Federation, arrived: Dict[str, Tuple[float, Any]], aggregator) -> Any:
    local_models = {a: p[1] for a, p in arrived.items() if p[1] is not None}
    everything: Dict[str, Any] = {}
    for part in fed.all_gather_object(local_models):
        everything.update(part)
    models = [everything[a] for a in sorted(everything)]
    if not models:
        return None
    agg = aggregator.aggregate(models)
    for a in arrived:
        if a in fed.local_nodes:
            fed.local_nodes[a].learner.set_model(agg)
    return agg
