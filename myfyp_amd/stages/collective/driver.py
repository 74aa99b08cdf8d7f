"""Lock-step round driver for co-located collective peers (host fast path).

With the fused MLP engine a whole federated round costs the GPU ~2 ms, while eight co-located peer
threads crossing two gang barriers per round spend comparable time just handing the GIL and the
barrier locks to each other. When every co-located peer is a fused-engine learner of one group
(no training callbacks, no workflow hooks) and the aggregator is sample-weighted averaging or
topology neighbour mixing (``fused_round.eligible``), the
peer threads therefore hand the remaining rounds to ONE driver thread (the last to arrive) and
sleep until their experiment ends. The driver executes, per round and for all local peers, exactly
what the collective stages would — Train/WaitAggregatedModels (one fused round: evaluation of every
trainer, the grouped local epoch(s), FedAvg collective, round hooks), GossipModel, RoundFinished
(aggregator reset, round counter, checkpoint) and the next vote (one all-gather) — and records the
same stage names in every peer's ``learning_workflow.history``. Collective call order per round is
identical to the threaded path, so ranks may mix the two.

Reference stage semantics: ``stages/base_node/{vote_train_set,train,gossip_model,round_finished}_stage.py``.
"""

from __future__ import annotations

import os
import threading
import time
from typing import Any, Dict

from myfyp_amd.management.checkpoint import maybe_checkpoint
from myfyp_amd.management.logger import logger
from myfyp_amd.management.tracing import mark
from myfyp_amd.parallel import weights_plane
from myfyp_amd.settings import Settings
from myfyp_amd.utils.lockcheck import make_lock
from myfyp_amd.stages.base_node.vote_train_set_stage import make_votes, tally_votes
from myfyp_amd.stages.collective import fused_round


def eligible(f, aggregator) -> bool:
    """Decided by the vote leader (so every co-located peer takes the same path)."""
    if not Settings.ROUND_DRIVER or not fused_round.eligible(f, aggregator):
        return False
    for a in f.local_order:
        node = f.local_nodes.get(a)
        if node is not None and getattr(node.learning_workflow, "hooks", None):
            return False  # fault injection / tracing hooks need the per-stage threaded path
    return True


class _Member:
    __slots__ = ("kw", "done", "error")

    def __init__(self, kw: Dict[str, Any]) -> None:
        self.kw = kw
        self.done = threading.Event()
        self.error: BaseException | None = None


class RoundDriver:
    """One per :class:`~myfyp_amd.parallel.federation.Federation`."""

    def __init__(self, f) -> None:
        self.f = f
        self.lock = make_lock("RoundDriver.members")
        self.members: Dict[str, _Member] = {}
        self.active = False

    # ------------------------------------------------------------------ membership
    def _claim(self) -> bool:
        with self.lock:
            expected = {a for a in self.f.local_order if a in self.f.local_nodes}
            if self.active or not self.members or not expected.issubset(self.members):
                return False
            self.active = True
            return True

    def enter(self, kw: Dict[str, Any]) -> None:
        """Called by each local peer thread right after this round's vote. Returns when the peer's
        experiment is over (its workflow then ends)."""
        state = kw["state"]
        m = _Member(kw)
        with self.lock:
            self.members[state.addr] = m
        while not m.done.is_set():
            if self._claim():
                members = dict(self.members)
                try:
                    prof_path = os.environ.get("MYFYP_PROFILE_DRIVER")
                    if prof_path:  # diagnostics: cProfile of the driver thread (host cost per round)
                        import cProfile

                        prof = cProfile.Profile()
                        try:
                            prof.runcall(self._drive, members)
                        finally:
                            prof.dump_stats(prof_path)
                    else:
                        self._drive(members)
                except BaseException as e:  # surfaced in every peer's learning thread
                    for mm in members.values():
                        mm.error = e
                finally:
                    for mm in members.values():
                        mm.done.set()
                    with self.lock:
                        for a in members:
                            self.members.pop(a, None)
                        self.active = False
                break
            if m.done.wait(timeout=0.5):
                break
            if state.round is None and not self.active:  # stopped while waiting for the others
                with self.lock:
                    self.members.pop(state.addr, None)
                return
        if m.error is not None:
            raise m.error

    # ------------------------------------------------------------------ the round loop
    def _drive(self, members: Dict[str, _Member]) -> None:
        f = self.f

        def live() -> Dict[str, _Member]:
            return {a: m for a, m in members.items() if a in f.local_nodes and m.kw["state"].round is not None}

        def history(m: _Member, name: str) -> None:
            m.kw["node"].learning_workflow.history.append(name)

        while True:
            cur = live()
            if not cur:
                return
            t0 = time.time()
            c0 = time.thread_time()  # host CPU time of this thread (excludes blocking waits)
            mark("driver_round")
            states = {a: m.kw["state"] for a, m in cur.items()}
            round_ = next(iter(states.values())).round
            train_set = list(next(iter(states.values())).train_set)
            trainers = [a for a in cur if a in train_set]
            # ---- TrainStage / WaitAggregatedModelsStage: one fused round for every local peer. The
            # launches go first, the per-peer bookkeeping after them: when the GPU is idle (the first
            # round, or after a host synchronisation) it waits for nothing else
            reqs = {a: cur[a].kw["learner"].fit_request() for a in trainers}
            out: Dict[str, Any] = {}
            mark("driver:launch")
            if trainers:
                has_test = {a for a in trainers if (d := cur[a].kw["learner"].data) is not None and d.get_num_samples(train=False) > 0}
                out = fused_round.run_groups(f, trainers, lambda a: cur[a].kw["learner"]._engine.slot, lambda a: cur[a].kw["learner"]._engine.group,
                                             reqs, has_test)
            snaps, n = {}, {}
            for a, m in cur.items():
                history(m, "TrainStage" if a in trainers else "WaitAggregatedModelsStage")
                snaps[a] = logger.experiment_snapshot(a)
                if a in trainers:
                    m.kw["aggregator"].set_nodes_to_aggregate(train_set)
                    n[a] = m.kw["learner"].num_train_samples()
            mark("driver:aggregate")
            total = next(iter(states.values())).total_rounds
            aggregator = next(iter(cur.values())).kw["aggregator"]
            fused_round.aggregate(f, {a: (n.get(a, 0), None) for a in cur}, aggregator, final=total is None or round_ + 1 >= total)
            for hook in list(f.round_hooks):
                hook(round_, f)
            mark("driver:results")
            for a, m in cur.items():
                lr = m.kw["learner"]
                if a in out:
                    ev, fit = out[a]
                    if ev is not None:
                        lr._evaluate_done(ev, snaps[a])
                    steps, mean_loss = fused_round.fit_result(fit)
                    lr.global_step += steps
                    lr._fit_done(steps, mean_loss, reqs[a][0])
                model = lr.get_model()
                model.set_contribution(train_set or [a], max(1, model.num_samples))
            # ---- GossipModelStage (no-op after the all-reduce) and RoundFinishedStage
            mark("driver:finish")
            final = []
            for a, m in cur.items():
                st = m.kw["state"]
                history(m, "GossipModelStage")
                history(m, "RoundFinishedStage")
                m.kw["aggregator"].clear()
                st.increase_round()
                logger.round_finished(a)
                if st.round is None or st.total_rounds is None:
                    raise ValueError("Round or total rounds not set.")
                maybe_checkpoint(st, m.kw["learner"])
                if st.round >= st.total_rounds:
                    final.append(a)
            logger.log_timing(next(iter(cur)), "driver_round", time.time() - t0)
            logger.log_timing(next(iter(cur)), "driver_round_cpu", time.thread_time() - c0)
            if final:
                self._finish({a: cur[a] for a in final})
                if len(final) == len(cur):
                    return
            # ---- VoteTrainSetStage of the next round: one all-gather of every local peer's votes
            cur = live()
            if not cur:
                return
            mark("driver:vote")
            votes = {}
            for a, m in cur.items():
                history(m, "VoteTrainSetStage")
                st = m.kw["state"]
                logger.round_started(a, st.experiment)
                votes[a] = make_votes(a, f.all_peers(), st.round)
            allv = weights_plane.gather_votes(f, votes)
            if getattr(aggregator, "all_peers_train", False):  # NeighborAvg: every live peer trains
                train_set = sorted(allv, key=lambda a: f.all_peers().index(a))
            else:
                train_set = tally_votes(allv)
            for a, m in cur.items():
                m.kw["state"].train_set = list(train_set)
            for hook in list(f.round_start_hooks):
                hook(next(iter(cur.values())).kw["state"].round, f)

    def _finish(self, done: Dict[str, _Member]) -> None:
        """Last round's RoundFinishedStage tail: final evaluation, state reset, experiment end."""
        from myfyp_amd.stages.collective._common import set_gang_expectations

        set_gang_expectations(self.f, set(), None)
        self.f.confirm_collectives()  # the last round's all-reduce, before the final evaluation reads the rows
        pend = {}
        slots = {a: m.kw["learner"]._engine.slot for a, m in done.items()}
        with_test = {a for a, m in done.items() if m.kw["learner"].data is not None and m.kw["learner"].data.get_num_samples(train=False) > 0}
        evs = {}
        by_group: Dict[int, Any] = {}
        for a in with_test:
            g = done[a].kw["learner"]._engine.group
            by_group.setdefault(id(g), (g, []))[1].append(a)
        for g, addrs in by_group.values():
            res = g._run_eval_batch({slots[a]: () for a in addrs})
            for a in addrs:
                evs[slots[a], id(g)] = res[slots[a]]
        for a, m in done.items():
            if a in with_test:
                pend[a] = m.kw["learner"]._evaluate_done(evs[slots[a], id(m.kw["learner"]._engine.group)], logger.experiment_snapshot(a))
        for a, m in done.items():
            results = pend[a].result() if a in pend else {}
            logger.info(a, f"📈 Final evaluation: {results}")
            m.kw["state"].clear()
            logger.experiment_finished(a)
