"""Noise floor of the CNN engine A/B tests (tests/test_cnn_engine_gpu.py): for each opt-in path
(env flag), the update distance (cosine, relative norm) between two default runs and between the
default and the opt-in run, at several batch / step configurations. Prints one line per case."""
import os
import sys
import threading

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_cnn_engine_gpu import _make_learners  # noqa: E402

from myfyp_amd.models import ResNet18  # noqa: E402


def run(flag, val, seed, n_train, batch):
    os.environ[flag] = val
    learners, _, _ = _make_learners(lambda i: ResNet18(seed=seed + i), 2, n_train, 16, batch, 0.05, momentum=0.9, wd=5e-4)
    g = learners[0]._engine.group
    p0 = [lr_.flat_params().detach().clone() for lr_ in learners]
    ths = [threading.Thread(target=lr_.fit) for lr_ in learners]
    [t.start() for t in ths]
    [t.join() for t in ths]
    torch.cuda.synchronize()
    loss = float(g.stat.view(g.capacity, 4)[0, 0])
    return [lr_.flat_params().detach().clone() - q for lr_, q in zip(learners, p0)], loss


def dist(xs, ys):
    return [(round(float(F.cosine_similarity(a, b, dim=0)), 5), round(float((a - b).norm() / b.norm()), 5)) for a, b in zip(xs, ys)]


for flag, seed in (("MYFYP_CNN_FUSE_BN", 70), ("MYFYP_CNN_FUSE_FIN", 110), ("MYFYP_CNN_S2_FWD", 90)):
    for n_train, batch in ((16, 16), (64, 64), (128, 64)):
        u1, l1 = run(flag, "0", seed, n_train, batch)
        u2, l2 = run(flag, "0", seed, n_train, batch)
        f, lf = run(flag, "1", seed, n_train, batch)
        os.environ[flag] = "0"
        print(f"{flag} n={n_train} B={batch}: floor {dist(u2, u1)} opt-in {dist(f, u1)} loss {l1:.5f} {l2:.5f} {lf:.5f}", flush=True)
