"""Round-level weight collectives executed by a local gang leader (see ``federation.py``).

All functions receive ``arrived: {addr: payload}`` for the co-located peers that reached the gang
and run identically on every rank (same call order ⇒ matching RCCL collectives).
"""

from __future__ import annotations

import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from myfyp_amd import ops
from myfyp_amd.management.tracing import traced
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
    """Every peer adopts the initiator's weights: local copy + one RCCL broadcast per tensor."""
    learners = {a: fed.local_nodes[a].learner for a in arrived if a in fed.local_nodes}
    fed.sync_members()
    src_rank = fed.peers.get(initiator, min(fed.members))
    ref_addr = initiator if initiator in learners else next(iter(learners))
    src = state_tensors(learners[ref_addr])
    bufs = [t.detach().clone() for t in src]
    for t in bufs:
        fed.broadcast_(t, src_rank)
    with torch.no_grad():
        for a, lr in learners.items():
            for dst, s in zip(state_tensors(lr), bufs):
                dst.copy_(s)


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
@traced("aggregate_mean")
def aggregate_mean(fed: Federation, arrived: Dict[str, Tuple[float, Any]]) -> Tuple[float, List[str]]:
    """Sample-weighted mean of the trainers' models (weight 0 for non-trainers), result into every
    local peer. One local weighted reduction kernel + one all-reduce + one broadcast kernel."""
    t0 = time.perf_counter()
    fed.sync_members()  # a rank may have lost its last peer since the vote: agree on the survivors
    addrs = [a for a in arrived if a in fed.local_nodes]  # a peer may die after arriving
    learners = [fed.local_nodes[a].learner for a in addrs]
    weights = [float(arrived[a][0]) for a in addrs]
    contributors = [a for a, w in zip(addrs, weights) if w > 0]
    group = _stacked_group(learners)
    dev = learners[0].flat_params().device
    if group is not None and dev.type == "cuda":
        # one native reduction kernel (weights as kernel arguments) -> RCCL all-reduce over the
        # n + 1 floats (weighted sum | Σw) -> one native normalise-and-broadcast kernel; no host
        # tensor traffic and nothing the host waits on
        w = np.zeros(group.capacity, dtype=np.float32)
        mask = np.zeros(group.capacity, dtype=np.float32)
        for lr, wt in zip(learners, weights):
            w[lr._engine.slot] = wt
            mask[lr._engine.slot] = 1.0
        n = group.numel
        fast = ops.fast_lib()
        stream = torch.cuda.current_stream(dev).cuda_stream
        if fed.solo:  # nothing to all-reduce: weighted mean and write-back in one launch
            ops.check(fast.myfyp_fedavg_stacked_local(group.params.data_ptr(), group.capacity, n, group.S, w.ctypes.data, mask.ctypes.data, stream),
                      "fedavg_local")
        else:
            buf = group.fedavg_buffer()
            ops.check(fast.myfyp_fedavg_stacked_reduce(buf.data_ptr(), group.params.data_ptr(), group.capacity, n, group.S, w.ctypes.data, stream), "fedavg_reduce")
            fed.all_reduce_(buf)
            ops.check(fast.myfyp_fedavg_stacked_apply(group.params.data_ptr(), buf.data_ptr(), group.capacity, n, group.S, mask.ctypes.data, stream), "fedavg_apply")
        total_w = float(sum(weights))  # local share; the global Σw stays on the device (buf[n])
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
        states = [state_tensors(lr) for lr in learners]
        flat = torch.cat([torch.cat([t.reshape(-1).float() for t in st]) for st in states[:1]])
        n = flat.numel()
        acc = torch.zeros(n + 1, dtype=torch.float32, device=dev)
        for st, wt in zip(states, weights):
            if wt > 0:
                acc[:n].add_(torch.cat([t.reshape(-1).float() for t in st]), alpha=wt)
        acc[n] = sum(weights)
        fed.all_reduce_(acc)
        total_w = float(acc[n])
        avg = acc[:n] / max(total_w, 1e-12)
        with torch.no_grad():
            for st in states:
                off = 0
                for t in st:
                    t.copy_(avg[off : off + t.numel()].view_as(t).to(t.dtype))
                    off += t.numel()
    fed.record("aggregate", time.perf_counter() - t0)
    return total_w, contributors


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
    fed.sync_members()
    peers = fed.all_peers()
    index = {a: i for i, a in enumerate(peers)}
    w = aggregator.mixing_matrix(len(peers))
    local = [a for a in peers if a in arrived and a in fed.local_nodes]
    if not local:
        fed.record("aggregate", time.perf_counter() - t0)
        return []
    learners = [fed.local_nodes[a].learner for a in local]
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
        for req in dist.batch_isend_irecv(ops_):
            req.wait()
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
    fed.sync_members()
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
    fed.record("aggregate", time.perf_counter() - t0)


@traced("aggregate_median")
def aggregate_median(fed: Federation, arrived: Dict[str, Tuple[float, Any]]) -> None:
    """Coordinate-wise median of the trainers' models on the device (``fedmedian.py:56-62``):
    the local trainers' flat rows are packed into a [k_max, n] buffer, ONE all-gather over the live
    ranks (RCCL) collects every trainer's row, and ONE ``k_coordinate_median<K>`` launch (sorting
    network in registers, <= 16 models) writes the result into every local peer. With a single
    rank the kernel reads the live rows directly (no packing copy)."""
    t0 = time.perf_counter()
    fed.sync_members()
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
        fed.record("aggregate", time.perf_counter() - t0)
        return
    import torch.distributed as dist

    ref = rows_of(addrs[0])
    n = ref.numel()
    send = torch.zeros(kmax, n, dtype=torch.float32, device=ref.device)
    for i, a in enumerate(trainers):
        send[i].copy_(rows_of(a))
    recv = torch.empty(len(counts) * kmax, n, dtype=torch.float32, device=ref.device)
    dist.all_gather_into_tensor(recv, send, group=fed.group)
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
    fed.record("aggregate", time.perf_counter() - t0)


def aggregate_generic(fed: Federation, arrived: Dict[str, Tuple[float, Any]], aggregator) -> Any:
    """Any aggregator: all-gather the trainers' wire models and reduce identically on every rank."""
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
