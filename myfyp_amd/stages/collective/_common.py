"""Helpers shared by the collective stages."""

from typing import Optional

from myfyp_amd.parallel.federation import Federation


def fed() -> Federation:
    return Federation.get()


def local_slot(node) -> Optional[int]:
    eng = getattr(node.learner, "_engine", None)
    return None if eng is None else eng.slot


def set_gang_expectations(f: Federation, fit_addrs, eval_addrs) -> None:
    """Tell fused-engine gangs exactly which co-located peers will call fit/evaluate."""
    groups = {}
    for a in f.local_order:
        node = f.local_nodes.get(a)
        eng = getattr(node.learner, "_engine", None) if node is not None else None
        if eng is not None:
            groups.setdefault(id(eng.group), (eng.group, set(), set()))
            g, fs, es = groups[id(eng.group)]
            if a in fit_addrs:
                fs.add(eng.slot)
            if eval_addrs is None or a in eval_addrs:
                es.add(eng.slot)
    for g, fs, es in groups.values():
        g.expect(fit_slots=fs, eval_slots=es if eval_addrs is not None else None)
