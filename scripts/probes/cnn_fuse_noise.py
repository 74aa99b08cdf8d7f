import os, sys, threading
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch, torch.nn.functional as F
import test_cnn_engine_gpu as T
from myfyp_amd.models import ResNet18
res = {}
for tag, fuse in (("u1", "0"), ("u2", "0"), ("f1", "1"), ("f2", "1")):
    os.environ["MYFYP_CNN_FUSE_BN"] = fuse
    learners, _, _ = T._make_learners(lambda i: ResNet18(seed=70 + i), 2, 16, 16, 16, 0.05, momentum=0.9, wd=5e-4)
    p0 = [l.flat_params().detach().clone() for l in learners]
    ths = [threading.Thread(target=l.fit) for l in learners]; [t.start() for t in ths]; [t.join() for t in ths]
    res[tag] = [l.flat_params().detach().clone() - q for l, q in zip(learners, p0)]
def cmp(a, b):
    return [(round(float(F.cosine_similarity(x, y, dim=0)), 5), round(float((x - y).norm() / y.norm()), 4)) for x, y in zip(res[a], res[b])]
print("u1 vs u2", cmp("u1", "u2")); print("f1 vs f2", cmp("f1", "f2")); print("f1 vs u1", cmp("f1", "u1"))
