"""Reference module layout of the PyTorch integration (``p2pfl/learning/frameworks/pytorch/``).

Lightning is not part of this stack: the MI355X learner drives the GPU directly (HBM-resident
partitions, fused HIP optimizer/engine kernels, hipGraph replay). These modules give reference
user code its import paths and class names on top of :mod:`myfyp_amd.learning.frameworks.torch`.
"""
