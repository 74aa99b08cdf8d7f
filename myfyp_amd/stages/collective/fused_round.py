"""One gang operation per round for co-located fused-engine peers: evaluate + fit + FedAvg.

The collective workflow normally crosses three barriers per round after the vote (evaluation gang,
fit gang, aggregation gang), each waking every co-located peer thread. When the vote leader finds
that every local peer is a fused-engine learner of one group without training callbacks and the
aggregator is sample-weighted averaging or topology neighbour mixing, the train / wait stages instead
join ONE gang whose leader enqueues, in stream order, the evaluation of every trainer, the grouped
local epoch(s) and the weight collective (FedAvg, or the NeighborAvg mix). Each peer thread then only files its own results (metrics are logged when the
device results land). Observable behaviour — stage history, metrics, contributions, the FedAvg
result — is that of the three-gang path (``train_stage.py`` / ``wait_agg_models_stage.py``;
reference ``stages/base_node/train_stage.py:44-100``).
"""

from __future__ import annotations

import time

from myfyp_amd.management.logger import logger
from myfyp_amd.parallel import weights_plane
from myfyp_amd.parallel.pending import Pending
from myfyp_amd.settings import Settings
from myfyp_amd.stages.collective._common import fed


def fit_result(fit):
    """(steps, mean train loss) of a group fit result: the MLP engine returns (steps, Pending of
    (loss, acc)) resolved asynchronously; the CNN engine (steps, loss, acc) as host floats."""
    if isinstance(fit[1], Pending):
        return fit[0], fit[1].map(lambda v: v[0])
    return fit[0], float(fit[1])


def eligible(f, aggregator) -> bool:
    """Decided once per round by the vote leader, so every co-located peer takes the same path."""
    if not Settings.FUSED_ROUND or getattr(aggregator, "collective_kind", None) not in ("mean", "neighbor"):
        return False
    groups: dict = {}
    for a in f.local_order:
        node = f.local_nodes.get(a)
        if node is None:
            continue
        lr = node.learner
        eng = getattr(lr, "_engine", None)
        if eng is None or getattr(lr, "callbacks", None) or not hasattr(lr, "fit_request"):
            return False
        groups.setdefault(getattr(lr, "mesh_rank", None), set()).add(id(eng.group))
    # one engine group, or (device mesh) one group per mesh rank
    if f.mesh is None:
        return len(groups) == 1 and all(len(v) == 1 for v in groups.values())
    return bool(groups) and all(len(v) == 1 for v in groups.values())


def run_groups(f, trainers, slot_of, group_of, reqs, with_test):
    """Enqueue the evaluation and the local epoch(s) of every trainer, one engine group at a time
    (one group per device of a mesh; each group's launches go to its own device's stream, so the
    devices run concurrently while this thread moves on). Returns {addr: (eval, fit)}."""
    by_group: dict = {}
    for a in trainers:
        g = group_of(a)
        by_group.setdefault(id(g), (g, []))[1].append(a)
    out = {}
    for g, addrs in by_group.values():
        evs = g._run_eval_batch({slot_of(a): () for a in addrs if a in with_test})
        fits = g._run_fit_batch({slot_of(a): reqs[a] for a in addrs})
        for a in addrs:
            out[a] = (evs.get(slot_of(a)), fits[slot_of(a)])
    return out


def aggregate(f, arrived, aggregator, final: bool) -> None:
    """The round's weight collective for an eligible aggregator: FedAvg (sample-weighted mean) or
    topology neighbour mixing (``NeighborAvg``)."""
    if getattr(aggregator, "collective_kind", None) == "neighbor":
        weights_plane.aggregate_neighbors(f, arrived, aggregator)
    else:
        weights_plane.aggregate_mean(f, arrived, final=final)


def join(state, learner, aggregator, trainer: bool) -> None:
    f = fed()
    t0 = time.time()
    snap = logger.experiment_snapshot(state.addr)
    req = learner.fit_request() if trainer else None
    n = learner.num_train_samples() if trainer else 0
    has_test = trainer and learner.data is not None and learner.data.get_num_samples(train=False) > 0
    round_ = state.round
    final = state.total_rounds is None or round_ + 1 >= state.total_rounds

    def leader(arrived):
        addrs = [a for a in arrived if a in f.local_nodes]  # a peer may die after arriving
        trainers = [a for a in addrs if arrived[a][0]]
        out = {}
        if trainers:
            out = run_groups(f, trainers, lambda a: f.local_nodes[a].learner._engine.slot, lambda a: f.local_nodes[a].learner._engine.group,
                             {a: arrived[a][2] for a in trainers}, {a for a in trainers if arrived[a][3]})
        aggregate(f, {a: (arrived[a][1], None) for a in addrs}, aggregator, final)
        for hook in list(f.round_hooks):
            hook(round_, f)
        return out

    res = f.gang_run(state.addr, (trainer, n, req, has_test), leader)
    if trainer:
        ev, fit = res[state.addr]
        if ev is not None:
            learner._evaluate_done(ev, snap)
        steps, mean_loss = fit_result(fit)
        learner.global_step += steps
        learner._fit_done(steps, mean_loss, req[0])
    model = learner.get_model()
    model.set_contribution(list(state.train_set) or [state.addr], max(1, model.num_samples))
    logger.log_timing(state.addr, "fused_round", time.time() - t0)
