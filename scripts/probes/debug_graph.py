"""Eager vs graph-replayed CNN engine fits: loss / accuracy trajectories."""
import os, sys, threading
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from test_cnn_engine_gpu import _make_learners
from myfyp_amd.models import LeNet5, ResNet18
arch = sys.argv[1] if len(sys.argv) > 1 else "lenet"
for eager in (True, False):
    fn = (lambda i: LeNet5(seed=40 + i)) if arch == "lenet" else (lambda i: ResNet18(seed=40 + i))
    learners, _, _ = _make_learners(fn, 2, 512, 256, 64, 0.05 if arch == "lenet" else 0.05, momentum=0.9)
    g = learners[0]._engine.group
    g.eager = eager
    for it in range(4):
        res = [None, None]
        ths = [threading.Thread(target=lambda i=i: res.__setitem__(i, learners[i].fit())) for i in range(2)]
        [t.start() for t in ths]; [t.join() for t in ths]
        st = g.stat.view(g.capacity, 4)[:2].tolist()
        ev = learners[0].evaluate()
        p = learners[0].flat_params()
        print(f"eager={eager} fit{it} stat={st} eval={ev['test_loss']:.4f}/{ev['test_metric']:.3f} |w|={float(p.norm()):.3f} nan={bool(torch.isnan(p).any())} graphs={len(g._graphs)}", flush=True)
