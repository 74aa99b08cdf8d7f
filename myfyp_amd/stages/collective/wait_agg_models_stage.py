"""Collective wait (parity target: ``stages/base_node/wait_agg_models_stage.py:40-67``).

A non-trainer contributes weight 0 to the same all-reduce, so collective membership never changes
while the FedAvg result still only averages the train set (SURVEY §7.4 hard part 1).
"""

from typing import Optional, Type

from myfyp_amd.parallel import weights_plane
from myfyp_amd.stages.collective._common import fed
from myfyp_amd.stages.stage import Stage
from myfyp_amd.stages.stage_factory import StageFactory


def join_aggregation(state, learner, aggregator, trainer: bool) -> None:
    f = fed()
    kind = getattr(aggregator, "collective_kind", None)
    model = learner.get_model()
    n = model.num_samples if trainer else 0
    wire = None
    on_device = kind in weights_plane.DEVICE_KINDS and hasattr(learner, "flat_params")
    if trainer and not on_device:
        wire = model.build_copy(params=model.get_parameters(), num_samples=model.num_samples, contributors=list(model.contributors), additional_info=dict(model.additional_info))
    round_ = state.round
    final = state.total_rounds is None or round_ + 1 >= state.total_rounds

    def leader(arrived):
        device_path = kind in ("scaffold", "median") and _agree_device_path(f, kind, arrived)
        if kind in ("scaffold", "median") and not device_path:
            arrived = _with_wire_models(f, arrived)
        if kind == "mean":
            total, contributors = weights_plane.aggregate_mean(f, arrived, final=final)
            extra = getattr(aggregator, "proximal_mu", None)
        elif kind == "neighbor":
            weights_plane.aggregate_neighbors(f, arrived, aggregator)
            extra = None
        elif kind == "scaffold" and device_path:
            weights_plane.aggregate_scaffold(f, arrived, aggregator)
            extra = None
        elif kind == "median" and device_path:
            weights_plane.aggregate_median(f, arrived)
            extra = None
        else:
            weights_plane.aggregate_generic(f, arrived, aggregator)
            extra = None
        for hook in list(f.round_hooks):
            hook(round_, f)
        return extra

    mu = f.gang_run(state.addr, (n, wire), leader)
    if mu is not None:
        model.add_info("fedprox", {"mu": mu})
        learner.update_callbacks_with_model_info()
    model.set_contribution(list(state.train_set) or [state.addr], max(1, model.num_samples))


def _agree_device_path(f, kind: str, arrived) -> bool:
    """SCAFFOLD / FedMedian reduce on the device only when EVERY rank's peers are device learners
    (flat parameter buffers): the ranks agree on it through one control-plane gather, so all of
    them issue the same collectives (a rank whose local peers happen to be non-trainers cannot
    tell from its own, empty, payloads)."""
    local_ok = all(hasattr(f.local_nodes[a].learner, "flat_params") for a in arrived if a in f.local_nodes)
    return all(f.all_gather_object(bool(local_ok)))


def _with_wire_models(f, arrived):
    """Generic path after the device path was voted down: local trainers that skipped building a
    wire model (they expected the device path) build it now."""
    out = {}
    for a, p in arrived.items():
        if p[0] and p[1] is None and a in f.local_nodes:
            model = f.local_nodes[a].learner.get_model()
            wire = model.build_copy(params=model.get_parameters(), num_samples=model.num_samples, contributors=list(model.contributors),
                                    additional_info=dict(model.additional_info))
            p = (p[0], wire)
        out[a] = p
    return out


class WaitAggregatedModelsStage(Stage):
    @staticmethod
    def name() -> str:
        return "WaitAggregatedModelsStage"

    @staticmethod
    def execute(state=None, communication_protocol=None, learner=None, aggregator=None, **kwargs) -> Optional[Type[Stage]]:
        if state is None or communication_protocol is None or learner is None or aggregator is None:
            raise Exception("Invalid parameters on WaitAggregatedModelsStage.")
        if state.round is None:
            return None
        if getattr(state, "fused_round", False):
            from myfyp_amd.stages.collective import fused_round

            fused_round.join(state, learner, aggregator, trainer=False)
        else:
            join_aggregation(state, learner, aggregator, trainer=False)
        return StageFactory.get_stage("GossipModelStage", "collective")
