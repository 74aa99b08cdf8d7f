"""Grouped CNN engine (LeNet-5 / ResNet-18): co-located peers trained by one sequence of HIP launches.

BASELINE configs 3-5 train CNNs on CIFAR-shaped data; the reference has no CNN at all. Like the MLP
engine (:mod:`myfyp_amd.parallel.mlp_engine`), every peer of one architecture/batch size on a device
gets a slot in stacked buffers and every kernel covers all peers through ``grid.z``:

* parameters live in one ``[capacity, S]`` fp32 buffer laid out ``[trainable params | BN running
  mean | BN running var]`` — the peers' ``nn.Module`` parameters *and* BN buffers are views into
  their row (wire format / ``state_dict`` unchanged; FedAvg over the stacked rows averages BN
  statistics too, like the reference's ``state_dict`` averaging);
* activations are NHWC bf16 (channels padded to a multiple of 8); each conv/fc weight has one bf16
  shadow ``Wf[Cout][R][S][Cin]`` (the forward B operand; the dgrad reads it N-contiguous through the
  LDS transpose read) and an fp32 gradient in the same layout, both handled by one fused
  optimizer kernel that maps between the GEMM layout and the torch-order master row in LDS;
* a train step is: input gather/convert → per conv: implicit-GEMM MFMA conv with BN partial sums
  fused in its epilogue → BN finalize → BN apply (+residual) + ReLU → … → avg-pool → fc →
  log-softmax/NLL (+dlogits) → backward (BN reduce/finalize/apply, dgrad conv with the residual
  gradient added in its epilogue, wgrad conv with transposed LDS reads) → SGD + shadow refresh;
* a whole local epoch is captured once into a HIP graph (``torch.cuda.CUDAGraph``) and replayed.

Numerics: bf16 activations/MFMA operands, fp32 accumulation, fp32 master weights, BN statistics and
optimizer state; torch SGD (momentum, weight decay, fresh optimizer per ``fit``) and torch
BatchNorm (biased batch variance for normalisation, unbiased running variance, momentum 0.1).
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, List, Optional, Set, Tuple

import numpy as np
import torch

from myfyp_amd.ops import _native
from myfyp_amd.parallel.mlp_engine import _Gang
from myfyp_amd.parallel.pending import Resolver
from myfyp_amd.settings import Settings

c_void_p, c_int, c_int64, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float


class ConvGemmArgs(ctypes.Structure):
    _fields_ = [
        ("src", c_void_p), ("src_ps", c_int64), ("src_h", c_int), ("src_w", c_int), ("src_c", c_int),
        ("out_h", c_int), ("out_w", c_int), ("R", c_int), ("S", c_int), ("stride", c_int), ("pad", c_int),
        ("wt", c_void_p), ("wt_ps", c_int64), ("ncol", c_int), ("ncol_valid", c_int),
        ("out", c_void_p), ("out_ps", c_int64), ("bias", c_void_p), ("bias_ps", c_int64),
        ("resid", c_void_p), ("resid_ps", c_int64), ("relu", c_int), ("stats", c_void_p), ("stats_ps", c_int64),
        ("nbatch", c_void_p), ("max_batch", c_int), ("pro_ss", c_void_p), ("pro_ss_ps", c_int64),
        ("bnb_mask", c_void_p), ("bnb_mask_ps", c_int64), ("bnb_y0", c_void_p), ("bnb_y0_ps", c_int64),
        ("bnb_y1", c_void_p), ("bnb_y1_ps", c_int64), ("bnb_ms0", c_void_p), ("bnb_ms1", c_void_p),
        ("bnb_part0", c_void_p), ("bnb_part1", c_void_p), ("bnb_part_ps", c_int64), ("stats_rows", c_int),
        ("bnb_rows", c_int), ("bnb_mask_ss", c_void_p), ("bnb_mask_ss_ps", c_int64),
        ("fin_cnt", c_void_p), ("fin_gamma0", c_void_p), ("fin_gamma1", c_void_p), ("fin_beta", c_void_p), ("fin_param_ps", c_int64),
        ("fin_rmean", c_void_p), ("fin_rvar", c_void_p), ("fin_run_ps", c_int64), ("fin_ss", c_void_p), ("fin_ms", c_void_p),
        ("fin_dgamma0", c_void_p), ("fin_dbeta0", c_void_p), ("fin_dgamma1", c_void_p), ("fin_dbeta1", c_void_p),
        ("fin_coef0", c_void_p), ("fin_coef1", c_void_p), ("fin_C0", c_int), ("fin_C1", c_int), ("fin_train", c_int),
        ("fin_eps", c_float), ("fin_momentum", c_float), ("fin_dbg", c_int),
    ]


class WgradArgs(ctypes.Structure):
    _fields_ = [
        ("dy", c_void_p), ("dy_ps", c_int64), ("x", c_void_p), ("x_ps", c_int64),
        ("H", c_int), ("W", c_int), ("x_c", c_int), ("Ho", c_int), ("Wo", c_int), ("dy_c", c_int),
        ("R", c_int), ("S", c_int), ("stride", c_int), ("pad", c_int),
        ("grad", c_void_p), ("grad_ps", c_int64), ("accumulate", c_int), ("k_per_split", c_int),
        ("nbatch", c_void_p), ("max_batch", c_int), ("pro_ss", c_void_p), ("pro_ss_ps", c_int64),
    ]


class LenetArgs(ctypes.Structure):
    """Mirror of ``LenetArgs`` (csrc/kernels/lenet_fused.h)."""

    _fields_ = [
        ("xs", c_void_p), ("ys", c_void_p), ("n_samples", c_void_p), ("perm", c_void_p), ("perm_ps", c_int64), ("offset", c_int), ("B", c_int),
        ("scale", c_float), ("shadow", c_void_p), ("shadow_ps", c_int64), ("w_c1", c_int64), ("w_c2", c_int64), ("w_f1", c_int64), ("w_f2", c_int64),
        ("w_f3", c_int64), ("params", c_void_p), ("params_ps", c_int64), ("b_c1", c_int64), ("b_c2", c_int64), ("b_f1", c_int64), ("b_f2", c_int64),
        ("b_f3", c_int64), ("gf", c_void_p), ("gf_ps", c_int64), ("g", c_void_p), ("g_ps", c_int64), ("act", c_void_p), ("act_ps", c_int64), ("part", c_void_p), ("part_ps", c_int64),
        ("wmaster", c_void_p), ("mom", c_void_p), ("shadow_rw", c_void_p), ("anchor", c_void_p), ("cg", c_void_p), ("cl", c_void_p),
        ("opt_kind", c_int), ("opt_lr", c_float), ("opt_beta1", c_float), ("opt_beta2", c_float), ("opt_eps", c_float), ("opt_wd", c_float),
        ("opt_momentum", c_float), ("opt_nesterov", c_int), ("opt_mu", c_float),
        ("t_c1", c_int64), ("t_c2", c_int64), ("t_f1", c_int64), ("t_f2", c_int64), ("t_f3", c_int64), ("f1_e2t", c_void_p),
        ("stats", c_void_p), ("confusion", c_void_p), ("nb", c_void_p), ("train", c_int),
    ]


LENET_ACT_W = 864  # per-image fc activation block of the fused LeNet step (lenet_fused.hip A_W)
LENET_IPW = 2  # images per workgroup of the fused LeNet step
LENET_PART_N = 4832  # floats per workgroup conv-gradient record (lenet_fused.hip PR_N)


class Segment(ctypes.Structure):
    _fields_ = [
        ("off", c_int64), ("n", c_int), ("kind", c_int), ("cout", c_int), ("cin", c_int), ("R", c_int), ("S", c_int),
        ("cp_in", c_int), ("cp_out", c_int), ("zero_after", c_int), ("pad_", c_int), ("wf_off", c_int64),
        ("e2t", c_void_p), ("t2e", c_void_p),
    ]


_SIGS = {
    "conv_gemm_launch": (c_int, [c_int, c_void_p, c_int, c_void_p]),
    "conv_set_dma": (c_int, [c_int]),
    "conv_set_dma_wgs": (c_int, [c_int]),
    "conv_set_wgrad_halo": (c_int, [c_int]),
    "conv_set_wgrad_pf": (c_int, [c_int]),
    "conv_set_fwd_halo": (c_int, [c_int]),
    "conv_gemm_stats_rows": (c_int, [c_int, c_int, c_int]),
    "conv_bnb_rows": (c_int, []),
    "conv_wgrad_launch": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "conv_wt_flip_launch": (c_int, [c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "conv_wt_flip_multi_launch": (c_int, [c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "conv_wt_flip_parity_launch": (c_int, [c_void_p, ctypes.c_longlong, c_void_p, ctypes.c_longlong, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "cnn_input_prep": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_void_p,
                               c_void_p, c_void_p]),
    "cnn_bn_finalize": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_int, c_float, c_float, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "cnn_bn_act": (c_int, [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_void_p]),
    "cnn_bn_bwd_reduce": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int64, c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p]),
    "cnn_bn_bwd_finalize": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]),
    "cnn_bn_bwd_apply": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p]),
    "conv_fin_words": (c_int, []),
    "conv_args_abi": (c_int, [c_void_p]),
    "conv_set_fin_debug": (c_int, [c_int]),
    "cnn_relu_bwd": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_void_p]),
    "cnn_colsum": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_int, c_void_p]),
    "cnn_maxpool2": (c_int, [c_int, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_void_p]),
    "cnn_avgpool": (c_int, [c_int, c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_int, c_void_p]),
    "cnn_xent": (c_int, [c_void_p, c_int64, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
    "cnn_opt_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_float, c_int, c_float,
                             c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_int, c_void_p]),
    "cnn_segment_size": (c_int, []),
    "lenet_fused_supported": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    "lenet_fused_step": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "lenet_args_size": (c_int, []),
}


def _lib():
    lib = _native.load(required=True)
    if not getattr(lib, "_cnn_sigs", False):
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        if lib.cnn_segment_size() != ctypes.sizeof(Segment):
            raise RuntimeError("Segment layout mismatch between Python and the native library")
        if lib.lenet_args_size() != ctypes.sizeof(LenetArgs):
            raise RuntimeError("LenetArgs layout mismatch between Python and the native library")
        abi = (ctypes.c_longlong * 4)()
        lib.conv_args_abi(abi)
        want = (ctypes.sizeof(ConvGemmArgs), ConvGemmArgs.fin_dbg.offset, ctypes.sizeof(WgradArgs), WgradArgs.pro_ss_ps.offset)
        if tuple(abi) != want:
            raise RuntimeError(f"ConvGemmArgs / WgradArgs layout mismatch between Python and the native library: {tuple(abi)} vs {want}")
        lib._cnn_sigs = True
    return lib


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _cp(c: int) -> int:
    return (c + 7) // 8 * 8


def _chk(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"CNN engine: {what} failed (rc={rc})")


# ------------------------------------------------------------------------------------------------
# architecture description
# ------------------------------------------------------------------------------------------------
class ConvL:
    """A conv (or fc = 1x1 conv on a 1x1 image) layer of the program."""

    def __init__(self, name: str, cin: int, cout: int, k: int, stride: int, pad: int, h: int, w: int, weight, bias=None, colmap=None) -> None:
        self.name, self.cin, self.cout, self.R, self.S, self.stride, self.pad = name, cin, cout, k, k, stride, pad
        self.h, self.w = h, w
        self.ho, self.wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
        self.cp_in, self.cp_out = _cp(cin), _cp(cout)
        self.weight, self.bias = weight, bias
        self.colmap = colmap  # torch input column -> engine channel (fc after NHWC flatten)


class BNL:
    def __init__(self, name: str, module: torch.nn.BatchNorm2d) -> None:
        self.name, self.module = name, module
        self.C = module.num_features
        self.Cp = _cp(self.C)
        self.eps, self.momentum = float(module.eps), float(module.momentum if module.momentum is not None else 0.1)


def arch_of(module: torch.nn.Module) -> Optional[str]:
    from myfyp_amd.models.cnn import LeNet5, ResNet18

    if isinstance(module, ResNet18):
        return "resnet18"
    if isinstance(module, LeNet5):
        return "lenet5"
    return None


def arch_key(module: torch.nn.Module) -> Optional[tuple]:
    a = arch_of(module)
    if a is None:
        return None
    shapes = tuple((n, tuple(p.shape)) for n, p in module.named_parameters())
    return (a, shapes, float(getattr(module, "input_scale", 1.0)), int(getattr(module, "image_size", 32)))


# ------------------------------------------------------------------------------------------------
# the group
# ------------------------------------------------------------------------------------------------
class CNNGroup:
    _groups: Dict[tuple, "CNNGroup"] = {}
    _lock = threading.Lock()

    @classmethod
    def get(cls, device: torch.device, module: torch.nn.Module, batch_size: int, tag=None) -> "CNNGroup":
        """``tag``: the peer's device-mesh rank (a virtual mesh puts several ranks on one GPU)."""
        key = (str(device), arch_key(module), batch_size, tag)
        with cls._lock:
            g = cls._groups.get(key)
            if g is None:
                g = cls(device, module, batch_size)
                g.mesh_rank = tag
                cls._groups[key] = g
            return g

    @classmethod
    def reset_all(cls) -> None:
        """Forget every group, releasing their captured graphs now (after the devices drain), not
        whenever the cyclic garbage collector reaches a dropped group: a torch CUDA graph destroyed
        from inside a collection, at an arbitrary point of later work, aborted a GPU test run."""
        with cls._lock:
            groups = list(cls._groups.values())
            cls._groups.clear()
        for dev in {g.device for g in groups if g.device.type == "cuda"}:
            torch.cuda.synchronize(dev)
        for g in groups:
            g.close()

    def __init__(self, device: torch.device, template: torch.nn.Module, batch_size: int, capacity: int = 8) -> None:
        self.device = device
        self.mesh_rank = None
        self.B = batch_size
        self.arch = arch_of(template)
        if device.type == "cuda":  # code objects loaded now, not at a first launch behind running kernels
            with torch.cuda.device(device):
                _native.warm_device(torch.cuda.current_device(), "cnn")
        self.lock = threading.RLock()
        self.resolver: Optional[Resolver] = None  # created on first use (device result copies)
        self.handles: Dict[int, "CNNEngineHandle"] = {}
        self.capacity = 0
        self.extras: Dict[str, torch.Tensor] = {}
        self.perm_fn = None
        self.eager = False
        # ResNet blocks, opt-in (MYFYP_CNN_FUSE_BN=1): BN1-apply + ReLU folded into conv2's forward /
        # wgrad operand prologues and its ReLU mask recomputed in the BN backward. Measured a net loss
        # on MI355X (+14 ms of 441 ms GPU time per profile, profiles/r2j_bn_prologue): the transform
        # is redone for each of the 9 im2col taps and every N tile, which costs more VALU in the
        # latency-bound conv loops than the k_bn_act pass it removes. Off by default.
        self.fuse_bn1 = os.environ.get("MYFYP_CNN_FUSE_BN", "0") == "1"
        # ResNet backward: the BN-backward column sums of a ReLU(BN) output are accumulated in the
        # epilogue of the dgrad that produces its gradient (k_bn_bwd_reduce skipped for those BNs;
        # MYFYP_CNN_FOLD_BNB=0: the separate reduce pass)
        self.fold_bnb = os.environ.get("MYFYP_CNN_FOLD_BNB", "1") != "0"
        # ResNet blocks whose conv2 runs on the patch-staged kernels (64 -> 64 channels, 3x3, stride
        # 1, 32-wide images: layer 1): BN1-apply + ReLU folded into conv2's forward / weight-gradient
        # patch staging (one transform per staged pixel, not per tap) and the dgrad's ReLU mask taken
        # from y1 — a1 is never written (MYFYP_CNN_HALO_BN1=0: materialise it as before)
        self.halo_bn1 = os.environ.get("MYFYP_CNN_HALO_BN1", "1") != "0"
        # BatchNorm finalize (batch statistics -> scale/shift, BN-backward sums -> apply coefficients)
        # run by the last workgroup of the conv that produced the sums (conv.hip conv_fin_tail)
        # instead of a k_bn_finalize / k_bn_bwd_finalize launch per BN. Opt-in (MYFYP_CNN_FUSE_FIN=1):
        # measured neutral on ResNet-18 in round 4 (2.536 vs 2.542 rounds/s, profiles/r4u_bn_fin_tail) —
        # the ~40 launches and their gaps go, but the last workgroup's serial chain (store drain, arrival
        # ticket, row gather, constants) lengthens every BN-producing conv by 2-12 us. With the
        # device-scope release / acquire fences the arrival ticket needs (round 5) it is 17 % slower:
        # 2.17-2.18 vs 2.62-2.64 rounds/s (profiles/r5_flip)
        self.fuse_fin = os.environ.get("MYFYP_CNN_FUSE_FIN", "0") == "1"
        # wgrad split-K target: workgroups per CU over all peers (more splits = more parallelism and
        # more fp32 atomics on the gradient)
        # stride-1 dgrad as a forward conv over dY with flipped weights (conv.hip MODE 4); 0 = MODE 3
        self.dgrad_fwd = os.environ.get("MYFYP_DGRAD_FWD", "1") != "0"
        # ResNet backward: every MODE-4 layer's weight flip in one launch at the start of the pass
        # (conv_wt_flip_multi_launch) instead of one before each dgrad (MYFYP_CNN_FLIP_BATCH=0):
        # 13 launches fewer per step, round rate the same (2.632 vs 2.630 rounds/s, profiles/r5_flip)
        self.flip_batch = os.environ.get("MYFYP_CNN_FLIP_BATCH", "1") != "0"
        self._flipped: frozenset = frozenset()
        self._flip_tables = None
        # ResNet backward: every weight gradient on a second stream (a branch of the captured step
        # graph), forked after its dY is written and joined before the optimizer. The dgrad chain
        # is the step's critical path; the weight gradients are leaves, so their workgroups fill
        # the CUs the chain's kernels leave idle (partial waves, epilogues, split-K atomic tails)
        # instead of running between them. MYFYP_CNN_WGRAD_STREAM=0: one stream
        self.wgrad_stream = os.environ.get("MYFYP_CNN_WGRAD_STREAM", "0") != "0"
        self._wg_side: Optional[torch.cuda.Stream] = None
        self.wgrad_tpc = int(os.environ.get("MYFYP_WGRAD_TPC", "2"))  # measured: 2 -> 75.6 ms wgrad, 4 -> 78.4, 8 -> 89.8 (scripts/probes/wgrad_tpc.sh)
        self.wgrad_tune = os.environ.get("MYFYP_WGRAD_TUNE", "1") != "0"  # per-layer split-K timed on the device (_tune_wgrad)
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._seen: set = set()
        self._data_version = 0
        self._bound_version = -1
        self.lenet_fused = False
        self._fit_seq = 0  # fit ids (interrupt_fit): one per fused fit, 0 = none
        self._slot_fit: Dict[int, int] = {}
        self._describe(template)
        self._alloc(capacity)
        self.fit_gang = _Gang(self._run_fit_batch, lambda: set(self.handles))
        self.eval_gang = _Gang(self._run_eval_batch, lambda: set(self.handles))

    # ------------------------------------------------------------------ description
    def _describe(self, m: torch.nn.Module) -> None:
        params = [p for p in m.parameters()]
        self.param_off: Dict[int, int] = {}
        off = 0
        for p in params:
            self.param_off[id(p)] = off
            off += p.numel()
        self.n_params = off
        self._param_names = {id(p): n for n, p in m.named_parameters()}
        self.bns: List[BNL] = []
        self.convs: List[ConvL] = []
        self.in_scale = float(getattr(m, "input_scale", 1.0))
        if self.arch == "resnet18":
            self.in_c = m.conv1.in_channels
            self.in_h = self.in_w = 32
            self._resnet_desc(m)
        else:
            self.in_c = m.conv1.in_channels
            self.in_h = self.in_w = int(getattr(m, "image_size", 32))
            self._lenet_desc(m)
        # BN running stats after the params: [rm(all BNs) | rv(all BNs)]
        self.bn_off: Dict[str, int] = {}
        o = 0
        for bn in self.bns:
            self.bn_off[bn.name] = o
            o += bn.C
        self.bn_total = o
        self.numel = self.n_params + 2 * self.bn_total
        self.S = (self.numel + 63) // 64 * 64
        # Wf shadows (bf16) and Wf-layout gradients (fp32) share offsets
        self.shadow_off: Dict[str, int] = {}
        so = 0
        for c in self.convs:
            self.shadow_off[c.name] = so
            so += c.cp_out * c.R * c.S * c.cp_in + 64
        self.shadow_numel = so

    def _off(self, p) -> int:
        return self.param_off[id(p)]

    def _resnet_desc(self, m) -> None:
        h = 32
        self.stem = ConvL("stem", m.conv1.in_channels, 64, 3, 1, 1, h, h, m.conv1.weight)
        self.stem_bn = BNL("stem_bn", m.bn1)
        self.convs.append(self.stem)
        self.bns.append(self.stem_bn)
        self.blocks = []
        for bi, blk in enumerate(m.layers):
            c1 = blk.conv1
            cv1 = ConvL(f"b{bi}c1", c1.in_channels, c1.out_channels, 3, c1.stride[0], 1, h, h, c1.weight)
            h2 = cv1.ho
            cv2 = ConvL(f"b{bi}c2", blk.conv2.in_channels, blk.conv2.out_channels, 3, 1, 1, h2, h2, blk.conv2.weight)
            bn1, bn2 = BNL(f"b{bi}bn1", blk.bn1), BNL(f"b{bi}bn2", blk.bn2)
            proj = None
            if len(blk.shortcut) > 0:
                sc, sbn = blk.shortcut[0], blk.shortcut[1]
                proj = (ConvL(f"b{bi}sc", sc.in_channels, sc.out_channels, 1, sc.stride[0], 0, h, h, sc.weight), BNL(f"b{bi}sbn", sbn))
            self.convs += [cv1, cv2] + ([proj[0]] if proj else [])
            self.bns += [bn1, bn2] + ([proj[1]] if proj else [])
            self.blocks.append((cv1, bn1, cv2, bn2, proj))
            h = h2
        self.final_hw = h * h
        self.fc = ConvL("fc", m.fc.in_features, m.fc.out_features, 1, 1, 0, 1, 1, m.fc.weight, m.fc.bias)
        self.convs.append(self.fc)
        self.n_classes = m.fc.out_features

    def _lenet_desc(self, m) -> None:
        h = self.in_h
        self.l_c1 = ConvL("c1", m.conv1.in_channels, m.conv1.out_channels, m.conv1.kernel_size[0], 1, 0, h, h, m.conv1.weight, m.conv1.bias)
        h1 = self.l_c1.ho // 2
        self.l_c2 = ConvL("c2", m.conv2.in_channels, m.conv2.out_channels, m.conv2.kernel_size[0], 1, 0, h1, h1, m.conv2.weight, m.conv2.bias)
        h2 = self.l_c2.ho // 2
        C2 = m.conv2.out_channels
        cp2 = _cp(C2)
        flat_in = h2 * h2 * cp2
        # torch flattens NCHW as (c, h, w); the engine's pooled tensor is (h, w, c) with padded c
        colmap = np.zeros(C2 * h2 * h2, dtype=np.int32)
        for c in range(C2):
            for y in range(h2):
                for x in range(h2):
                    colmap[(c * h2 + y) * h2 + x] = (y * h2 + x) * cp2 + c
        self.l_fc1 = ConvL("fc1", flat_in, m.fc1.out_features, 1, 1, 0, 1, 1, m.fc1.weight, m.fc1.bias, colmap=colmap)
        self.l_fc1.cin_torch = C2 * h2 * h2
        self.l_fc2 = ConvL("fc2", m.fc2.in_features, m.fc2.out_features, 1, 1, 0, 1, 1, m.fc2.weight, m.fc2.bias)
        self.l_fc3 = ConvL("fc3", m.fc3.in_features, m.fc3.out_features, 1, 1, 0, 1, 1, m.fc3.weight, m.fc3.bias)
        self.convs = [self.l_c1, self.l_c2, self.l_fc1, self.l_fc2, self.l_fc3]
        self.lenet_h = (h, h1, h2)
        self.n_classes = m.fc3.out_features
        # whole step in one fused kernel (lenet_fused.hip) when the shapes are the reference LeNet-5's
        self.lenet_fused = False
        if Settings.USE_FUSED_KERNELS and os.environ.get("MYFYP_LENET_FUSED", "1") != "0" and self.device.type == "cuda":
            self.lenet_fused = bool(_lib().lenet_fused_supported(self.in_c, h, m.conv1.out_channels, m.conv2.out_channels, m.fc1.out_features,
                                                                  m.fc2.out_features, m.fc3.out_features, self.B)) and self.B % LENET_IPW == 0

    # ------------------------------------------------------------------ buffers
    def _alloc(self, capacity: int) -> None:
        dev = self.device
        old = getattr(self, "params", None)
        params = torch.zeros(capacity, self.S, dtype=torch.float32, device=dev)
        if old is not None:
            params[: self.capacity].copy_(old)
        self.params = params
        self.grad = torch.zeros_like(params)
        self.mom = torch.zeros_like(params)
        self.shadow = torch.zeros(capacity, self.shadow_numel, dtype=torch.bfloat16, device=dev)
        self.gradf = torch.zeros(capacity, self.shadow_numel, dtype=torch.float32, device=dev)
        self.shadow_t = torch.zeros_like(self.shadow) if self.dgrad_fwd else None  # MODE 4 weights (k_conv_wt_flip)
        # interrupted fits: a stop word per slot in host-pinned memory (written by interrupt() while
        # the epoch runs, read by every step's input kernel) and the device copy of each slot's
        # current fit id (uploaded in stream order at the fit's start: a stale stop word never
        # matches a later fit)
        self._stop = torch.zeros(capacity, dtype=torch.int32, pin_memory=dev.type == "cuda")
        self._fit_id = torch.zeros(capacity, dtype=torch.int32, device=dev)
        self.s2_fwd = os.environ.get("MYFYP_CNN_S2_FWD", "0") == "1"  # MODE 5 stride-2 dgrads (see conv())
        self.capacity = capacity
        for slot, h in self.handles.items():
            h.retarget()
        self._acts: Dict[str, torch.Tensor] = {}
        self._graphs.clear()
        self._seen = set()
        self._tune_wgrad()
        self._build_segments()

    def _tune_wgrad(self) -> None:
        """Pick each ResNet wgrad layer's split-K count on the device (before the optimizer segments,
        whose zero-after flags follow it, and before any graph capture). The best split depends on
        the shape's workgroup count against the resident slots (a second, partial wave of workgroups
        nearly doubles a launch) and on the K-loop length per workgroup, in ways a formula tracked
        poorly: a sweep of the ResNet-18 shapes (profiles/r3z_wsplit) put the round-2 rule 1-18 %
        off the best per layer (layer-3 wgrad 155 us at 1 split, 132 us at 3). Candidates around
        that rule are timed on scratch operands of the layer's shape; MYFYP_WGRAD_TUNE=0 keeps the rule."""
        self._wsplit: Dict[str, Tuple[int, int]] = {}
        if not (self.wgrad_tune and self.arch == "resnet18" and self.device.type == "cuda" and Settings.USE_FUSED_KERNELS):
            return
        lib, P = _lib(), self.capacity
        s = torch.cuda.current_stream(self.device)
        cache: Dict[tuple, Tuple[int, int]] = {}
        for L in self.convs:
            if L.colmap is not None:
                continue
            key = (L.h, L.w, L.cp_in, L.cp_out, L.R, L.S, L.stride, L.pad)
            if key in cache:
                self._wsplit[L.name] = cache[key]
                continue
            M = self.B * L.ho * L.wo
            base = self._wgrad_split_rule(L)[1]
            # around the rule, plus a ladder up to 64 (the halo wgrad of the 64-channel layers wants one
            # workgroup per CU: 32 splits x 8 peers, off the rule's multiples)
            cands = sorted({max(1, min(64, int(round(base * f)))) for f in (0.5, 1, 1.5, 2, 3, 4)} | {1, 2, 4, 8, 16, 32, 64})
            x = torch.zeros(P, self.B * L.h * L.w * L.cp_in, dtype=torch.bfloat16, device=self.device)
            dy = torch.zeros(P, M * L.cp_out, dtype=torch.bfloat16, device=self.device)
            grad = torch.zeros(P, L.cp_out * L.R * L.S * L.cp_in, dtype=torch.float32, device=self.device)
            best, seen = None, set()
            for want in cands:
                k_per = max(64, ((M + want - 1) // want + 63) // 64 * 64)
                splits = (M + k_per - 1) // k_per
                if splits in seen:
                    continue
                seen.add(splits)
                a = WgradArgs()
                a.dy, a.dy_ps, a.x, a.x_ps = dy.data_ptr(), dy.shape[1], x.data_ptr(), x.shape[1]
                a.H, a.W, a.x_c, a.Ho, a.Wo, a.dy_c = L.h, L.w, L.cp_in, L.ho, L.wo, L.cp_out
                a.R, a.S, a.stride, a.pad = L.R, L.S, L.stride, L.pad
                a.grad, a.grad_ps, a.accumulate, a.k_per_split, a.max_batch = grad.data_ptr(), grad.shape[1], int(splits > 1), k_per, self.B
                for _ in range(2):
                    _chk(lib.conv_wgrad_launch(ctypes.byref(a), P, splits, s.cuda_stream), "wgrad tune")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(5):
                    _chk(lib.conv_wgrad_launch(ctypes.byref(a), P, splits, s.cuda_stream), "wgrad tune")
                e1.record(s)
                e1.synchronize()
                t = e0.elapsed_time(e1)
                if best is None or t < best[0]:
                    best = (t, (k_per, splits))
            cache[key] = best[1]
            self._wsplit[L.name] = best[1]
            del x, dy, grad

    def _build_segments(self) -> None:
        segs, work = [], []
        self._keep_colmaps = []
        for c in self.convs:
            e2t = t2e = 0
            if c.colmap is not None:  # fc after the NHWC flatten: engine channel <-> torch column maps
                inv = np.full(c.cp_in, -1, dtype=np.int32)
                inv[c.colmap] = np.arange(len(c.colmap), dtype=np.int32)
                te, tt = torch.from_numpy(inv).to(self.device), torch.from_numpy(np.asarray(c.colmap, dtype=np.int32)).to(self.device)
                self._keep_colmaps += [te, tt]
                e2t, t2e = te.data_ptr(), tt.data_ptr()
            cin_t = getattr(c, "cin_torch", c.cin)
            # LDS rows of k_opt_step (cnn_ops.hip SHADOW_MAX_ROW / GRAD_MAX_ROW)
            if cin_t * c.R * c.S + cin_t // 8 > 4608 + 64 or (c.cp_in + 4) * c.R * c.S > 9 * (512 + 4):
                raise ValueError(f"conv layer {c.name} too wide for the optimizer kernel (cin * R * S > 4608)")
            accumulate = int(self._wgrad_split(c)[1] > 1)
            if getattr(self, "lenet_fused", False) and c.name in ("c1", "c2"):
                accumulate = 1  # the fused step adds its per-workgroup conv gradients atomically
            work += [(len(segs), co) for co in range(c.cout)]
            segs.append(Segment(self._off(c.weight), c.weight.numel(), 1, c.cout, cin_t, c.R, c.S, c.cp_in, c.cp_out, accumulate, 0, self.shadow_off[c.name], e2t, t2e))
            if c.bias is not None:
                work += [(len(segs), k) for k in range((c.bias.numel() + 255) // 256)]
                segs.append(Segment(self._off(c.bias), c.bias.numel(), 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0))
        for bn in self.bns:
            for p in (bn.module.weight, bn.module.bias):
                work += [(len(segs), k) for k in range((p.numel() + 255) // 256)]
                segs.append(Segment(self._off(p), p.numel(), 0, 0, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0))
        arr = (Segment * len(segs))(*segs)
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.segs = raw.to(self.device)
        self.nseg = len(segs)
        self.work = torch.tensor(work, dtype=torch.int32).reshape(-1, 2).to(self.device)
        self.nwork = len(work)

    def act(self, name: str, rows: int, cp: int, dtype=torch.bfloat16) -> torch.Tensor:
        t = self._acts.get(name)
        if t is None:
            t = torch.zeros(self.capacity, rows * cp, dtype=dtype, device=self.device)
            self._acts[name] = t
        return t

    def fbuf(self, name: str, n: int) -> torch.Tensor:
        return self.act(name, n, 1, torch.float32)

    def ibuf(self, name: str, n: int) -> torch.Tensor:
        return self.act(name, n, 1, torch.int32)

    def attach(self, handle: "CNNEngineHandle") -> int:
        with self.lock:
            slot = next((i for i in range(self.capacity) if i not in self.handles), None)
            if slot is None:
                self._alloc(self.capacity * 2)
                slot = next(i for i in range(self.capacity) if i not in self.handles)
            self.handles[slot] = handle
            self._data_version += 1
            return slot

    def detach(self, slot: int) -> None:
        with self.lock:
            self.handles.pop(slot, None)
            self._data_version += 1
        self.fit_gang.poke()
        self.eval_gang.poke()

    def invalidate_data(self) -> None:
        with self.lock:
            self._data_version += 1

    def close(self) -> None:
        self._graphs.clear()

    def _extra_buffer(self, name: str) -> torch.Tensor:
        buf = self.extras.get(name)
        if buf is None or buf.shape[0] != self.capacity:
            buf = torch.zeros(self.capacity, self.S, dtype=torch.float32, device=self.device)
            self.extras[name] = buf
        return buf

    # ------------------------------------------------------------------ data binding
    def _bind_data(self) -> None:
        cap, dev = self.capacity, self.device
        self._keep = []
        xs, ys, ns, xts, yts, nts = [0] * cap, [0] * cap, [0] * cap, [0] * cap, [0] * cap, [0] * cap
        for slot, h in self.handles.items():
            (x, y), (xt, yt) = h.device_split(True), h.device_split(False)
            xs[slot], ys[slot], ns[slot] = x.data_ptr(), y.data_ptr(), x.shape[0]
            xts[slot], yts[slot], nts[slot] = xt.data_ptr(), yt.data_ptr(), xt.shape[0]
            self._keep += [x, y, xt, yt]
        self.n_train, self.n_test = ns, nts
        self.tab = {
            "xs": torch.tensor(xs, dtype=torch.int64, device=dev), "ys": torch.tensor(ys, dtype=torch.int64, device=dev),
            "n": torch.tensor(ns, dtype=torch.int32, device=dev), "xts": torch.tensor(xts, dtype=torch.int64, device=dev),
            "yts": torch.tensor(yts, dtype=torch.int64, device=dev), "nt": torch.tensor(nts, dtype=torch.int32, device=dev),
        }
        self.nmax = max(1, max(ns) if ns else 1)
        self.ntmax = max(1, max(nts) if nts else 1)
        self.perm = torch.zeros(cap, self.nmax, dtype=torch.int32, device=dev)
        self._perm_mask = torch.arange(self.nmax, device=dev).unsqueeze(0) >= torch.tensor(ns, device=dev).unsqueeze(1)
        self._graphs.clear()
        self._seen = set()

    def _ensure(self) -> None:
        if self._bound_version != self._data_version:
            self._bind_data()
            self._bound_version = self._data_version

    # ------------------------------------------------------------------ kernel wrappers
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def conv(self, L: ConvL, src: torch.Tensor, out: torch.Tensor, mode: int = 0, bias: bool = False, relu: bool = False, resid=None, stats=None,
             pro: Optional["BNL"] = None, bnb: Optional[tuple] = None, bnb_mask_bn: Optional["BNL"] = None, fin: Optional["BNL"] = None,
             train: bool = True, bnb_fin: bool = False) -> None:
        """``pro``: src holds that BatchNorm's input y; the conv reads relu(BN(y)) in its prologue.
        ``bnb`` (dgrad): ``(mask, [(bn, y), ...])`` — out is written as the ReLU-masked gradient g and
        the BN-backward sums of each listed BatchNorm (input y) accumulate in the epilogue; follow
        with ``bn_bwd(..., pre_reduced=True)``. ``bnb_mask_bn`` (with a None mask): the ReLU mask is
        relu(BN(y0)) > 0 of that BatchNorm, computed from y0 in the epilogue (the activation was
        never materialised). ``fin`` (forward): that BatchNorm's finalize runs in the conv's last
        workgroup (in place of ``bn_fin``; ``train`` False: from the running statistics).
        ``bnb_fin`` (dgrad with ``bnb``): the listed BatchNorms' backward finalize runs there too
        (then ``bn_bwd(..., pre_reduced=True, finalized=True)``)."""
        lib, P = _lib(), self.capacity
        shadow_f = self.shadow_off[L.name]
        a = ConvGemmArgs()
        # stride-1 dgrad as a forward conv over dY with flipped, transposed weights (conv.hip MODE 4):
        # the forward's K-contiguous weight panel instead of the transposed LDS reads of MODE 3
        fwd_dgrad = mode == 1 and L.stride == 1 and L.colmap is None and self.dgrad_fwd
        # stride-2 dgrad by parity class, each class a forward conv over dY with its flipped taps
        # (conv.hip MODE 5, LDS-DMA kernel only). Opt-in (MYFYP_CNN_S2_FWD=1): measured neutral — the
        # classes' K loops are 1-4 taps long, and the flip costs more than the gather it saves
        # (stride-2 dgrads 21.7 vs 20.3-22.1 ms per profiled run, profiles/r3z_conv_dma); with the
        # compile-time epilogues on both paths still 0.9 % slower (profiles/r4y_s2_parity_spec)
        par_dgrad = mode == 1 and L.stride == 2 and L.colmap is None and self.dgrad_fwd and self.s2_fwd and lib.conv_set_dma(-1) != 0
        if par_dgrad:
            wt = self.shadow_t.data_ptr() + 2 * shadow_f
            _chk(lib.conv_wt_flip_parity_launch(self.shadow.data_ptr() + 2 * shadow_f, self.shadow.shape[1], wt, self.shadow_t.shape[1], L.cp_out, L.cp_in,
                                                L.R, L.S, L.pad, P, self._stream()), f"wt parity flip {L.name}")
            a.src, a.src_h, a.src_w, a.src_c = src.data_ptr(), L.ho, L.wo, L.cp_out
            a.out_h, a.out_w = L.h, L.w
            a.wt = wt
            a.ncol, a.ncol_valid = L.cp_in, L.cin
        elif fwd_dgrad:
            wt = self.shadow_t.data_ptr() + 2 * shadow_f
            if L.name not in self._flipped:
                _chk(lib.conv_wt_flip_launch(self.shadow.data_ptr() + 2 * shadow_f, self.shadow.shape[1], wt, self.shadow_t.shape[1], L.cp_out, L.cp_in, L.R, L.S,
                                             P, self._stream()), f"wt flip {L.name}")
            a.src, a.src_h, a.src_w, a.src_c = src.data_ptr(), L.ho, L.wo, L.cp_out
            a.out_h, a.out_w = L.h, L.w
            a.wt = wt
            a.ncol, a.ncol_valid = L.cp_in, L.cin
        elif mode == 0:
            a.src, a.src_h, a.src_w, a.src_c = src.data_ptr(), L.h, L.w, L.cp_in
            a.out_h, a.out_w = L.ho, L.wo
            a.wt = self.shadow.data_ptr() + 2 * shadow_f
            a.ncol, a.ncol_valid = L.cp_out, L.cout
        else:
            a.src, a.src_h, a.src_w, a.src_c = src.data_ptr(), L.ho, L.wo, L.cp_out
            a.out_h, a.out_w = L.h, L.w
            a.wt = self.shadow.data_ptr() + 2 * shadow_f
            a.ncol, a.ncol_valid = L.cp_in, (L.cin if L.colmap is None else L.cp_in)
        a.src_ps, a.wt_ps = src.shape[1], self.shadow.shape[1]
        a.R, a.S, a.stride, a.pad = L.R, L.S, L.stride, (L.R - 1 - L.pad if fwd_dgrad else L.pad)
        a.out, a.out_ps = out.data_ptr(), out.shape[1]
        if bias and L.bias is not None:
            a.bias, a.bias_ps = self.params.data_ptr() + 4 * self._off(L.bias), self.params.shape[1]
        if resid is not None:
            a.resid, a.resid_ps = resid.data_ptr(), resid.shape[1]
        a.relu = int(relu)
        if stats is not None:
            a.stats, a.stats_ps = stats.data_ptr(), stats.shape[1]
            a.stats_rows = stats.shape[1] // (2 * a.ncol)
        a.nbatch, a.max_batch = self.nb.data_ptr(), self.B
        if pro is not None:
            ss = self.ss(pro)
            a.pro_ss, a.pro_ss_ps = ss.data_ptr(), ss.shape[1]
        if bnb is not None:
            mask, targets = bnb
            assert mode == 1 and 1 <= len(targets) <= 2 and all(bn.Cp == a.ncol for bn, _ in targets)
            if mask is not None:
                a.bnb_mask, a.bnb_mask_ps = mask.data_ptr(), mask.shape[1]
            elif bnb_mask_bn is not None:
                mss = self.ss(bnb_mask_bn)
                a.bnb_mask_ss, a.bnb_mask_ss_ps = mss.data_ptr(), mss.shape[1]
            (bn0, y0), rest = targets[0], targets[1:]
            nr = lib.conv_bnb_rows()
            a.bnb_rows = nr
            part0 = self.fbuf(f"bnsum_{bn0.name}", nr * 2 * bn0.Cp)
            a.bnb_y0, a.bnb_y0_ps, a.bnb_ms0, a.bnb_part0, a.bnb_part_ps = y0.data_ptr(), y0.shape[1], self.ms(bn0).data_ptr(), part0.data_ptr(), part0.shape[1]
            if rest:
                bn1_, y1_ = rest[0]
                a.bnb_y1, a.bnb_y1_ps, a.bnb_ms1 = y1_.data_ptr(), y1_.shape[1], self.ms(bn1_).data_ptr()
                a.bnb_part1 = self.fbuf(f"bnsum_{bn1_.name}", nr * 2 * bn1_.Cp).data_ptr()
            if bnb_fin:
                gb, pb = self.grad.data_ptr(), self.params.data_ptr()
                a.fin_cnt = self.ibuf(f"fincnt_b_{L.name}", lib.conv_fin_words()).data_ptr()
                a.fin_param_ps = self.params.shape[1]
                assert self.grad.shape[1] == self.params.shape[1]
                for i, (bn_, _) in enumerate(targets):
                    w_, b_ = self._off(bn_.module.weight), self._off(bn_.module.bias)
                    setattr(a, f"fin_gamma{i}", pb + 4 * w_)
                    setattr(a, f"fin_dgamma{i}", gb + 4 * w_)
                    setattr(a, f"fin_dbeta{i}", gb + 4 * b_)
                    setattr(a, f"fin_coef{i}", self.fbuf(f"bncoef_{bn_.name}", 3 * bn_.Cp).data_ptr())
                    setattr(a, f"fin_C{i}", bn_.C)
        if fin is not None:
            assert mode == 0 and fin.Cp == a.ncol
            base = self.params.data_ptr()
            ro = self.n_params + self.bn_off[fin.name]
            a.fin_cnt = self.ibuf(f"fincnt_f_{L.name}", lib.conv_fin_words()).data_ptr()
            a.fin_gamma0, a.fin_beta = base + 4 * self._off(fin.module.weight), base + 4 * self._off(fin.module.bias)
            a.fin_param_ps = a.fin_run_ps = self.params.shape[1]
            a.fin_rmean, a.fin_rvar = base + 4 * ro, base + 4 * (ro + self.bn_total)
            a.fin_ss, a.fin_ms = self.ss(fin).data_ptr(), self.ms(fin).data_ptr()
            a.fin_C0, a.fin_train, a.fin_eps, a.fin_momentum = fin.C, int(train), fin.eps, fin.momentum
        _chk(lib.conv_gemm_launch(5 if par_dgrad else (4 if fwd_dgrad else mode), ctypes.byref(a), P, self._stream()), f"conv {L.name} mode {mode}")

    def _wgrad_split(self, L: ConvL) -> Tuple[int, int]:
        """(pixels per split, splits): the device-tuned choice (``_tune_wgrad``) or the rule."""
        tuned = getattr(self, "_wsplit", {}).get(L.name)
        return tuned if tuned is not None else self._wgrad_split_rule(L)

    def _wgrad_split_rule(self, L: ConvL) -> Tuple[int, int]:
        """(pixels per split, splits): split the pixel (K) dimension only until ~wgrad_tpc tiles per CU exist."""
        M = self.B * L.ho * L.wo
        ncol = L.R * L.S * L.cp_in
        tiles = ((L.cp_out + 127) // 128) * ((ncol + 127) // 128)
        want = max(1, (self.wgrad_tpc * 256) // max(1, tiles * self.capacity))
        k_per = max(64, ((M + want - 1) // want + 63) // 64 * 64)
        return k_per, (M + k_per - 1) // k_per

    def wgrad(self, L: ConvL, dy: torch.Tensor, x: torch.Tensor, pro: Optional["BNL"] = None) -> None:
        lib, P = _lib(), self.capacity
        a = WgradArgs()
        a.dy, a.dy_ps, a.x, a.x_ps = dy.data_ptr(), dy.shape[1], x.data_ptr(), x.shape[1]
        a.H, a.W, a.x_c, a.Ho, a.Wo, a.dy_c = L.h, L.w, L.cp_in, L.ho, L.wo, L.cp_out
        a.R, a.S, a.stride, a.pad = L.R, L.S, L.stride, L.pad
        a.grad, a.grad_ps = self.gradf.data_ptr() + 4 * self.shadow_off[L.name], self.gradf.shape[1]
        k_per, splits = self._wgrad_split(L)
        a.accumulate = int(splits > 1)  # must match the segment's zero_after (the optimizer re-zeroes)
        a.k_per_split, a.nbatch, a.max_batch = k_per, self.nb.data_ptr(), self.B
        if pro is not None:
            ss = self.ss(pro)
            a.pro_ss, a.pro_ss_ps = ss.data_ptr(), ss.shape[1]
        _chk(lib.conv_wgrad_launch(ctypes.byref(a), P, splits, self._stream()), f"wgrad {L.name}")

    def bn_fin(self, bn: BNL, stats: torch.Tensor, rows: int, hw: int, train: bool) -> None:
        lib, P = _lib(), self.capacity
        g, b = bn.module.weight, bn.module.bias
        ro = self.n_params + self.bn_off[bn.name]
        base = self.params.data_ptr()
        _chk(lib.cnn_bn_finalize(
            _p(stats) if stats is not None else None, stats.shape[1] if stats is not None else 0, rows, self.nb.data_ptr(), hw,
            base + 4 * self._off(g), base + 4 * self._off(b), self.params.shape[1], base + 4 * ro, base + 4 * (ro + self.bn_total), self.params.shape[1],
            bn.C, bn.Cp, bn.eps, bn.momentum, int(train), self.ss(bn).data_ptr(), self.ms(bn).data_ptr(), P, self._stream()), f"bn_fin {bn.name}")

    def conv_bn(self, L: ConvL, src, out, bn: BNL, st, hw: int, train: bool, **kw) -> None:
        """Forward conv producing BatchNorm ``bn``'s input, then that BN's finalize: in the conv's
        last workgroup (``fuse_fin``) or as its own launch."""
        if self.fuse_fin and self.device.type == "cuda":
            self.conv(L, src, out, stats=st, fin=bn, train=train, **kw)
        else:
            self.conv(L, src, out, stats=st, **kw)
            self.bn_fin(bn, st, st.shape[1] // (2 * L.cp_out) if st is not None else 0, hw, train)

    def _bn1_in_halo(self, c2: "ConvL") -> bool:
        """conv2 of this block takes BN1 + ReLU in its patch staging (k_conv_fwd_halo /
        k_conv_wgrad_halo shapes; the halo kernels must be on)."""
        if not (self.halo_bn1 and not self.fuse_bn1 and self.device.type == "cuda"):
            return False
        lib = _lib()
        on = lib.conv_set_fwd_halo(-1) != 0 and lib.conv_set_wgrad_halo(-1) != 0
        return (on and c2.cp_in == 64 and c2.cp_out == 64 and c2.R == 3 and c2.S == 3 and c2.stride == 1 and c2.pad == 1 and c2.w == 32
                and c2.h * 32 % 256 == 0 and c2.colmap is None)

    def ss(self, bn: BNL) -> torch.Tensor:
        return self.fbuf(f"ss_{bn.name}", 2 * bn.Cp)

    def ms(self, bn: BNL) -> torch.Tensor:
        return self.fbuf(f"ms_{bn.name}", 2 * bn.Cp)

    def bn_act(self, bn: BNL, y, out, hw, relu=True, res=None, y2=None, bn2: Optional[BNL] = None) -> None:
        lib, P = _lib(), self.capacity
        _chk(lib.cnn_bn_act(y.data_ptr(), y.shape[1], self.ss(bn).data_ptr(), _p(res), res.shape[1] if res is not None else 0, _p(y2),
                            y2.shape[1] if y2 is not None else 0, self.ss(bn2).data_ptr() if bn2 is not None else None, int(relu), self.nb.data_ptr(),
                            self.B * hw, hw, bn.Cp, out.data_ptr(), out.shape[1], P, self._stream()), f"bn_act {bn.name}")

    def bn_bwd(self, bn: BNL, dz, mask, y, dy_out, hw, gout=None, mask_from_y: bool = False, pre_reduced: bool = False, finalized: bool = False) -> None:
        """``mask_from_y``: the ReLU after this BN was never materialised; its mask is y*sc + sh > 0.
        ``pre_reduced``: dz is already the masked gradient g and its sums were accumulated by the
        producing dgrad's epilogue (``conv(..., bnb=...)``): only finalize + apply run.
        ``finalized``: that dgrad's last workgroup also ran the finalize (``conv(..., bnb_fin=True)``):
        only the apply runs."""
        lib, P = _lib(), self.capacity
        mss = self.ss(bn).data_ptr() if mask_from_y else None
        nblk = max(1, min(128, (self.B * hw + 255) // 256))
        nr = lib.conv_bnb_rows()  # accumulator rows (spread atomics), summed and re-zeroed by the finalize
        part = self.fbuf(f"bnsum_{bn.name}", nr * 2 * bn.Cp)
        coef = self.fbuf(f"bncoef_{bn.name}", 3 * bn.Cp)
        if pre_reduced:
            assert mask is None and gout is None and not mask_from_y
        else:
            _chk(lib.cnn_bn_bwd_reduce(dz.data_ptr(), dz.shape[1], _p(mask), mask.shape[1] if mask is not None else 0, y.data_ptr(), y.shape[1],
                                       self.ms(bn).data_ptr(), self.nb.data_ptr(), hw, bn.Cp, part.data_ptr(), part.shape[1], nblk, _p(gout),
                                       gout.shape[1] if gout is not None else 0, P, self._stream(), mss), f"bn_bwd_reduce {bn.name}")
        assert not finalized or pre_reduced
        gbase = self.grad.data_ptr()
        if not finalized:
            _chk(lib.cnn_bn_bwd_finalize(part.data_ptr(), part.shape[1], nr, self.nb.data_ptr(), hw, self.params.data_ptr() + 4 * self._off(bn.module.weight),
                                         self.params.shape[1], self.ms(bn).data_ptr(), gbase + 4 * self._off(bn.module.weight),
                                         gbase + 4 * self._off(bn.module.bias), bn.C, bn.Cp, coef.data_ptr(), P, self._stream()), f"bn_bwd_finalize {bn.name}")
        _chk(lib.cnn_bn_bwd_apply(dz.data_ptr(), dz.shape[1], _p(mask), mask.shape[1] if mask is not None else 0, y.data_ptr(), y.shape[1],
                                  self.ms(bn).data_ptr(), coef.data_ptr(), self.nb.data_ptr(), self.B * hw, hw, bn.Cp, dy_out.data_ptr(),
                                  dy_out.shape[1], P, self._stream(), mss), f"bn_bwd_apply {bn.name}")

    def relu_bwd(self, dz, mask, out, hw, cp) -> None:
        _chk(_lib().cnn_relu_bwd(dz.data_ptr(), dz.shape[1], mask.data_ptr(), mask.shape[1], self.nb.data_ptr(), self.B * hw, hw, cp, out.data_ptr(),
                                 out.shape[1], self.capacity, self._stream()), "relu_bwd")

    def bias_grad(self, L: ConvL, dy, hw) -> None:
        nblk = max(1, min(64, (self.B * hw + 255) // 256))
        _chk(_lib().cnn_colsum(dy.data_ptr(), dy.shape[1], self.nb.data_ptr(), hw, L.cp_out, L.cout, self.grad.data_ptr() + 4 * self._off(L.bias),
                               self.grad.shape[1], nblk, self.capacity, self._stream()), f"bias_grad {L.name}")

    # ------------------------------------------------------------------ programs
    def _prep(self, train: bool, offset: int) -> torch.Tensor:
        lib, P, B = _lib(), self.capacity, self.B
        cp0 = _cp(self.in_c)
        x0 = self.act("x0", B * self.in_h * self.in_w, cp0)
        t = self.tab
        perm = self.perm if train else None
        _chk(lib.cnn_input_prep(_p(t["xs"] if train else t["xts"]), _p(t["ys"] if train else t["yts"]), _p(t["n"] if train else t["nt"]), _p(perm),
                                self.nmax if train else 0, offset, B, self.in_h, self.in_w, self.in_c, cp0, self.in_scale, x0.data_ptr(), x0.shape[1],
                                self.labels.data_ptr(), self.nb.data_ptr(), P, self._stream(), _p(self._stop) if train else None,
                                _p(self._fit_id) if train else None), "input_prep")
        return x0

    def _forward_resnet(self, x0: torch.Tensor, train: bool) -> torch.Tensor:
        B = self.B
        L, bn = self.stem, self.stem_bn
        hw = L.ho * L.wo
        y = self.act("y_stem", B * hw, L.cp_out)
        st = self.fbuf("st_stem", _lib().conv_gemm_stats_rows(B, L.ho, L.wo) * 2 * L.cp_out) if train else None
        self.conv_bn(L, x0, y, bn, st, hw, train)
        a = self.act("a_stem", B * hw, L.cp_out)
        self.bn_act(bn, y, a, hw)
        for bi, (c1, bn1, c2, bn2, proj) in enumerate(self.blocks):
            a_in = a
            hw1 = c1.ho * c1.wo
            rows1 = _lib().conv_gemm_stats_rows(B, c1.ho, c1.wo)
            y1 = self.act(f"y1_{bi}", B * hw1, c1.cp_out)
            st1 = self.fbuf(f"st1_{bi}", rows1 * 2 * c1.cp_out) if train else None
            self.conv_bn(c1, a_in, y1, bn1, st1, hw1, train)
            y2 = self.act(f"y2_{bi}", B * hw1, c2.cp_out)
            st2 = self.fbuf(f"st2_{bi}", rows1 * 2 * c2.cp_out) if train else None
            if self.fuse_bn1 or self._bn1_in_halo(c2):  # BN1-apply + ReLU in conv2's operand prologue (a1 never written)
                self.conv_bn(c2, y1, y2, bn2, st2, hw1, train, pro=bn1)
            else:
                a1 = self.act(f"a1_{bi}", B * hw1, c1.cp_out)
                self.bn_act(bn1, y1, a1, hw1)
                self.conv_bn(c2, a1, y2, bn2, st2, hw1, train)
            a = self.act(f"a2_{bi}", B * hw1, c2.cp_out)
            if proj is not None:
                cs, bns = proj
                ys = self.act(f"ys_{bi}", B * hw1, cs.cp_out)
                sts = self.fbuf(f"sts_{bi}", rows1 * 2 * cs.cp_out) if train else None
                self.conv_bn(cs, a_in, ys, bns, sts, hw1, train)
                self.bn_act(bn2, y2, a, hw1, y2=ys, bn2=bns)
            else:
                self.bn_act(bn2, y2, a, hw1, res=a_in)
        pooled = self.act("pooled", B, self.fc.cp_in)
        _chk(_lib().cnn_avgpool(0, a.data_ptr(), a.shape[1], self.nb.data_ptr(), B, self.final_hw, self.fc.cp_in, pooled.data_ptr(), pooled.shape[1],
                                self.capacity, self._stream()), "avgpool")
        logits = self.act("logits", B, self.fc.cp_out)
        self.conv(self.fc, pooled, logits, bias=True)
        self._last_act = a
        return logits

    def _flip_all(self, layers) -> None:
        """One launch flipping the MODE-4 weights of every layer in ``layers`` (``conv`` then skips
        their per-layer flips until the pass ends)."""
        if self._flip_tables is None:
            todo = [L for L in layers if L.stride == 1 and L.colmap is None]
            offs = (ctypes.c_longlong * len(todo))(*[self.shadow_off[L.name] for L in todo])
            dims = (c_int * (4 * len(todo)))(*[v for L in todo for v in (L.cp_out, L.cp_in, L.R, L.S)])
            self._flip_tables = (frozenset(L.name for L in todo), len(todo), offs, dims)
        names, n, offs, dims = self._flip_tables
        if n:
            _chk(_lib().conv_wt_flip_multi_launch(self.shadow.data_ptr(), self.shadow.shape[1], self.shadow_t.data_ptr(), self.shadow_t.shape[1], n, offs,
                                                  dims, self.capacity, self._stream()), "wt flip (all layers)")
        self._flipped = names

    def _backward_resnet(self, dlogits: torch.Tensor) -> None:
        batched = self.flip_batch and self.dgrad_fwd and self.shadow_t is not None
        if batched:
            self._flip_all([self.fc] + [c for blk in self.blocks for c in (blk[0], blk[2])])
        side = None
        if self.wgrad_stream and self.device.type == "cuda":
            if self._wg_side is None:
                self._wg_side = torch.cuda.Stream(self.device)
            side = self._wg_side
        self._wg_branch = side
        try:
            self._backward_resnet_pass(dlogits)
        finally:
            self._flipped = frozenset()
            self._wg_branch = None
            if side is not None:  # join: the optimizer reads every weight gradient
                torch.cuda.current_stream(self.device).wait_stream(side)

    def _wgrad_b(self, L: ConvL, dy: torch.Tensor, x: torch.Tensor, pro: Optional["BNL"] = None) -> None:
        """``wgrad`` on the backward's side stream when one is open (forked here: dY and x are final
        on the current stream; nothing the branch reads is written again before the join)."""
        side = getattr(self, "_wg_branch", None)
        if side is None:
            self.wgrad(L, dy, x, pro)
            return
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            self.wgrad(L, dy, x, pro)

    def _backward_resnet_pass(self, dlogits: torch.Tensor) -> None:
        B, lib = self.B, _lib()
        fc = self.fc
        pooled = self.act("pooled", B, fc.cp_in)
        dpooled = self.act("dpooled", B, fc.cp_in)
        self.conv(fc, dlogits, dpooled, mode=1)
        self._wgrad_b(fc, dlogits, pooled)
        self.bias_grad(fc, dlogits, 1)
        last = self.blocks[-1][2]
        hw = last.ho * last.wo
        d = self.act(f"d_out_{len(self.blocks) - 1}", B * hw, last.cp_out)
        _chk(lib.cnn_avgpool(1, dpooled.data_ptr(), dpooled.shape[1], self.nb.data_ptr(), B, self.final_hw, fc.cp_in, d.data_ptr(), d.shape[1],
                             self.capacity, self._stream()), "avgpool_bwd")
        fold = self.fold_bnb
        ff = self.fuse_fin and self.device.type == "cuda"  # pre-reduced BN sums are finalized by their dgrad too
        pre = False  # d is already the masked gradient of this block's output, its BN sums accumulated
        for bi in range(len(self.blocks) - 1, -1, -1):
            c1, bn1, c2, bn2, proj = self.blocks[bi]
            hw1 = c1.ho * c1.wo
            a_out = self.act(f"a2_{bi}", B * hw1, c2.cp_out)
            a_in = self.act(f"a2_{bi - 1}", B * c1.h * c1.w, c1.cp_in) if bi > 0 else self.act("a_stem", B * c1.h * c1.w, c1.cp_in)
            y1, y2 = self.act(f"y1_{bi}", B * hw1, c1.cp_out), self.act(f"y2_{bi}", B * hw1, c2.cp_out)
            halo1 = self._bn1_in_halo(c2)
            a1 = None if (self.fuse_bn1 or halo1) else self.act(f"a1_{bi}", B * hw1, c1.cp_out)
            dy2 = self.act(f"dy2_{bi}", B * hw1, c2.cp_out)
            d_in = self.act(f"d_out_{bi - 1}" if bi > 0 else "d_stem", B * c1.h * c1.w, c1.cp_in)
            mask_out = None if pre else a_out
            if proj is not None:
                cs, bns = proj
                ys = self.act(f"ys_{bi}", B * hw1, cs.cp_out)
                self.bn_bwd(bn2, d, mask_out, y2, dy2, hw1, pre_reduced=pre, finalized=pre and ff)
                dys = self.act(f"dys_{bi}", B * hw1, cs.cp_out)
                self.bn_bwd(bns, d, mask_out, ys, dys, hw1, pre_reduced=pre, finalized=pre and ff)
                dsc = self.act(f"dsc_{bi}", B * c1.h * c1.w, c1.cp_in)
                self.conv(cs, dys, dsc, mode=1)
                self._wgrad_b(cs, dys, a_in)
                resid = dsc
            elif pre:
                self.bn_bwd(bn2, d, None, y2, dy2, hw1, pre_reduced=True, finalized=ff)
                resid = d  # already the masked gradient g
            else:
                g = self.act(f"g_{bi}", B * hw1, c2.cp_out)
                self.bn_bwd(bn2, d, a_out, y2, dy2, hw1, gout=g)
                resid = g
            da1 = self.act(f"da1_{bi}", B * hw1, c1.cp_out)
            dy1 = self.act(f"dy1_{bi}", B * hw1, c1.cp_out)
            if halo1 and fold:  # a1 never written: mask from y1 in the dgrad epilogue, BN1 in the wgrad staging
                self.conv(c2, dy2, da1, mode=1, bnb=(None, [(bn1, y1)]), bnb_mask_bn=bn1, bnb_fin=ff)
                self._wgrad_b(c2, dy2, y1, pro=bn1)
                self.bn_bwd(bn1, da1, None, y1, dy1, hw1, pre_reduced=True, finalized=ff)
            elif self.fuse_bn1 or halo1:
                self.conv(c2, dy2, da1, mode=1)
                self._wgrad_b(c2, dy2, y1, pro=bn1)
                self.bn_bwd(bn1, da1, None, y1, dy1, hw1, mask_from_y=True)
            elif fold:
                self.conv(c2, dy2, da1, mode=1, bnb=(a1, [(bn1, y1)]), bnb_fin=ff)
                self._wgrad_b(c2, dy2, a1)
                self.bn_bwd(bn1, da1, None, y1, dy1, hw1, pre_reduced=True, finalized=ff)
            else:
                self.conv(c2, dy2, da1, mode=1)
                self._wgrad_b(c2, dy2, a1)
                self.bn_bwd(bn1, da1, a1, y1, dy1, hw1)
            bnb = None
            if fold:  # d_in is the gradient of the previous block's (or the stem's) ReLU(BN) output
                if bi > 0:
                    pc1, _, pc2, pbn2, pproj = self.blocks[bi - 1]
                    phw = pc1.ho * pc1.wo
                    tg = [(pbn2, self.act(f"y2_{bi - 1}", B * phw, pc2.cp_out))]
                    if pproj is not None:
                        tg.append((pproj[1], self.act(f"ys_{bi - 1}", B * phw, pproj[0].cp_out)))
                    bnb = (a_in, tg)
                else:
                    st = self.stem
                    bnb = (a_in, [(self.stem_bn, self.act("y_stem", B * st.ho * st.wo, st.cp_out))])
            self.conv(c1, dy1, d_in, mode=1, resid=resid, bnb=bnb, bnb_fin=ff and bnb is not None)
            self._wgrad_b(c1, dy1, a_in)
            d = d_in
            pre = bnb is not None
        L, bn = self.stem, self.stem_bn
        hw = L.ho * L.wo
        dys = self.act("dy_stem", B * hw, L.cp_out)
        if pre:
            self.bn_bwd(bn, d, None, self.act("y_stem", B * hw, L.cp_out), dys, hw, pre_reduced=True, finalized=ff)
        else:
            self.bn_bwd(bn, d, self.act("a_stem", B * hw, L.cp_out), self.act("y_stem", B * hw, L.cp_out), dys, hw)
        self._wgrad_b(L, dys, self.act("x0", B * self.in_h * self.in_w, _cp(self.in_c)))

    def _forward_lenet(self, x0: torch.Tensor, train: bool) -> torch.Tensor:
        B, lib, P = self.B, _lib(), self.capacity
        c1, c2, f1, f2, f3 = self.l_c1, self.l_c2, self.l_fc1, self.l_fc2, self.l_fc3
        h0, h1, h2 = self.lenet_h
        z1 = self.act("z1", B * c1.ho * c1.wo, c1.cp_out)
        self.conv(c1, x0, z1, bias=True, relu=True)
        p1 = self.act("p1", B * h1 * h1, c1.cp_out)
        _chk(lib.cnn_maxpool2(0, z1.data_ptr(), z1.shape[1], None, 0, self.nb.data_ptr(), B, c1.ho, c1.wo, c1.cp_out, p1.data_ptr(), p1.shape[1], P,
                              self._stream()), "maxpool1")
        z2 = self.act("z2", B * c2.ho * c2.wo, c2.cp_out)
        self.conv(c2, p1, z2, bias=True, relu=True)
        p2 = self.act("p2", B * h2 * h2, c2.cp_out)
        _chk(lib.cnn_maxpool2(0, z2.data_ptr(), z2.shape[1], None, 0, self.nb.data_ptr(), B, c2.ho, c2.wo, c2.cp_out, p2.data_ptr(), p2.shape[1], P,
                              self._stream()), "maxpool2")
        # p2 [B][h2][w2][cp2] is exactly fc1's [B][1][1][h2*w2*cp2] input
        z3 = self.act("z3", B, f1.cp_out)
        self.conv(f1, p2, z3, bias=True, relu=True)
        z4 = self.act("z4", B, f2.cp_out)
        self.conv(f2, z3, z4, bias=True, relu=True)
        logits = self.act("logits", B, f3.cp_out)
        self.conv(f3, z4, logits, bias=True)
        return logits

    def _backward_lenet(self, dlogits: torch.Tensor) -> None:
        B, lib, P = self.B, _lib(), self.capacity
        c1, c2, f1, f2, f3 = self.l_c1, self.l_c2, self.l_fc1, self.l_fc2, self.l_fc3
        h0, h1, h2 = self.lenet_h
        z4, z3 = self.act("z4", B, f2.cp_out), self.act("z3", B, f1.cp_out)
        p2, z2 = self.act("p2", B * h2 * h2, c2.cp_out), self.act("z2", B * c2.ho * c2.wo, c2.cp_out)
        p1, z1 = self.act("p1", B * h1 * h1, c1.cp_out), self.act("z1", B * c1.ho * c1.wo, c1.cp_out)
        x0 = self.act("x0", B * self.in_h * self.in_w, _cp(self.in_c))
        # fc3
        self.wgrad(f3, dlogits, z4)
        self.bias_grad(f3, dlogits, 1)
        dz4 = self.act("dz4", B, f2.cp_out)
        self.conv(f3, dlogits, dz4, mode=1)
        g4 = self.act("g4", B, f2.cp_out)
        self.relu_bwd(dz4, z4, g4, 1, f2.cp_out)
        self.wgrad(f2, g4, z3)
        self.bias_grad(f2, g4, 1)
        dz3 = self.act("dz3", B, f1.cp_out)
        self.conv(f2, g4, dz3, mode=1)
        g3 = self.act("g3", B, f1.cp_out)
        self.relu_bwd(dz3, z3, g3, 1, f1.cp_out)
        self.wgrad(f1, g3, p2)
        self.bias_grad(f1, g3, 1)
        dp2 = self.act("dp2", B * h2 * h2, c2.cp_out)
        self.conv(f1, g3, dp2, mode=1)
        dz2 = self.act("dz2", B * c2.ho * c2.wo, c2.cp_out)
        _chk(lib.cnn_maxpool2(1, z2.data_ptr(), z2.shape[1], dp2.data_ptr(), dp2.shape[1], self.nb.data_ptr(), B, c2.ho, c2.wo, c2.cp_out, dz2.data_ptr(),
                              dz2.shape[1], P, self._stream()), "maxpool2_bwd")
        g2 = self.act("g2", B * c2.ho * c2.wo, c2.cp_out)
        self.relu_bwd(dz2, z2, g2, c2.ho * c2.wo, c2.cp_out)
        self.wgrad(c2, g2, p1)
        self.bias_grad(c2, g2, c2.ho * c2.wo)
        dp1 = self.act("dp1", B * h1 * h1, c1.cp_out)
        self.conv(c2, g2, dp1, mode=1)
        dz1 = self.act("dz1", B * c1.ho * c1.wo, c1.cp_out)
        _chk(lib.cnn_maxpool2(1, z1.data_ptr(), z1.shape[1], dp1.data_ptr(), dp1.shape[1], self.nb.data_ptr(), B, c1.ho, c1.wo, c1.cp_out, dz1.data_ptr(),
                              dz1.shape[1], P, self._stream()), "maxpool1_bwd")
        g1 = self.act("g1", B * c1.ho * c1.wo, c1.cp_out)
        self.relu_bwd(dz1, z1, g1, c1.ho * c1.wo, c1.cp_out)
        self.wgrad(c1, g1, x0)
        self.bias_grad(c1, g1, c1.ho * c1.wo)

    def _xent(self, logits, train: bool) -> None:
        Lp = self.convs[-1].cp_out
        dl = self.act("dlogits", self.B, Lp) if train else None
        _chk(_lib().cnn_xent(logits.data_ptr(), logits.shape[1], Lp, self.n_classes, self.labels.data_ptr(), self.B, self.nb.data_ptr(),
                             self.stat.data_ptr(), None if train else self.conf.data_ptr(), _p(dl), dl.shape[1] if dl is not None else 0, self.capacity,
                             self._stream()), "xent")

    def _train_step(self, offset: int) -> None:
        if self.arch != "resnet18" and self.lenet_fused:
            self._lenet_fused(True, offset)  # forward, backward and the SGD step
            return
        x0 = self._prep(True, offset)
        if self.arch == "resnet18":
            logits = self._forward_resnet(x0, True)
            self._xent(logits, True)
            self._backward_resnet(self.act("dlogits", self.B, self.fc.cp_out))
        else:
            logits = self._forward_lenet(x0, True)
            self._xent(logits, True)
            self._backward_lenet(self.act("dlogits", self.B, self.l_fc3.cp_out))
        self._optimizer(update=True)

    def _lenet_fused(self, train: bool, offset: int) -> None:
        """One fused LeNet-5 step (train: forward + backward + gradients; eval: forward + loss /
        confusion) for every peer: ``lenet_fused.hip``."""
        t, P, B = self.tab, self.capacity, self.B
        a = LenetArgs()
        a.xs, a.ys, a.n_samples = _p(t["xs"] if train else t["xts"]), _p(t["ys"] if train else t["yts"]), _p(t["n"] if train else t["nt"])
        a.perm, a.perm_ps = (_p(self.perm), self.nmax) if train else (None, 0)
        a.offset, a.B, a.scale = offset, B, self.in_scale
        a.shadow, a.shadow_ps = self.shadow.data_ptr(), self.shadow.shape[1]
        so = self.shadow_off
        a.w_c1, a.w_c2, a.w_f1, a.w_f2, a.w_f3 = so["c1"], so["c2"], so["fc1"], so["fc2"], so["fc3"]
        a.params, a.params_ps = self.params.data_ptr(), self.params.shape[1]
        L = (self.l_c1, self.l_c2, self.l_fc1, self.l_fc2, self.l_fc3)
        a.b_c1, a.b_c2, a.b_f1, a.b_f2, a.b_f3 = (self._off(x.bias) for x in L)
        a.gf, a.gf_ps = self.gradf.data_ptr(), self.gradf.shape[1]
        a.g, a.g_ps = self.grad.data_ptr(), self.grad.shape[1]
        act = self.act("lenet_act", B * LENET_ACT_W, 1)
        a.act, a.act_ps = act.data_ptr(), act.shape[1]
        part = self.fbuf("lenet_part", (B // LENET_IPW) * LENET_PART_N)
        a.part, a.part_ps = part.data_ptr(), part.shape[1]
        a.stats, a.confusion, a.nb = self.stat.data_ptr(), None if train else self.conf.data_ptr(), self.nb.data_ptr()
        a.train = int(train)
        if train:  # SGD applied by the fc-gradient kernel where each gradient is produced (no k_opt_step)
            o = self._opt
            a.wmaster, a.mom, a.shadow_rw = self.params.data_ptr(), self.mom.data_ptr(), self.shadow.data_ptr()
            a.anchor, a.cg, a.cl = _p(o.get("anchor")), _p(o.get("cg")), _p(o.get("cl"))
            a.opt_kind, a.opt_lr, a.opt_beta1, a.opt_beta2, a.opt_eps = o["kind"], o["lr"], 0.9, 0.999, 1e-8
            a.opt_wd, a.opt_momentum, a.opt_nesterov, a.opt_mu = o["weight_decay"], o["momentum"], o["nesterov"], o["mu"]
            a.t_c1, a.t_c2, a.t_f1, a.t_f2, a.t_f3 = (self._off(x.weight) for x in L)
            a.f1_e2t = self._keep_colmaps[0].data_ptr()  # fc1 is the only layer with a column map (engine -> torch)
        _chk(_lib().lenet_fused_step(ctypes.byref(a), P, LENET_IPW, self._stream()), "lenet_fused_step")

    def _optimizer(self, update: bool) -> None:
        """SGD on the torch-order master rows + bf16 Wf shadow rows, one fused launch (update=False:
        shadow refresh only). Atomically accumulated gradients are re-zeroed as they are consumed."""
        o = self._opt
        _chk(_lib().cnn_opt_step(self.params.data_ptr(), self.grad.data_ptr(), self.mom.data_ptr(), self.params.shape[1], self.gradf.data_ptr(),
                                 self.gradf.shape[1], self.segs.data_ptr(), self.work.data_ptr(), self.nwork, o["kind"], o["lr"], o["momentum"],
                                 o["weight_decay"], o["nesterov"], o["mu"], _p(o.get("anchor")), _p(o.get("cg")), _p(o.get("cl")), int(update),
                                 self.shadow.data_ptr(), self.shadow.shape[1], self.nb.data_ptr() if update else None, self.capacity, self._stream()),
             "optimizer")

    def _shadow_sync(self) -> None:
        saved = getattr(self, "_opt", None)
        self._opt = {"kind": 1, "lr": 0.0, "momentum": 0.0, "weight_decay": 0.0, "nesterov": 0, "mu": 0.0}
        self._optimizer(update=False)
        if saved is not None:
            self._opt = saved

    # ------------------------------------------------------------------ batched fit / eval
    def _common_buffers(self) -> None:
        self.nb = self.ibuf("nb", 1)
        self.labels = self.ibuf("labels", self.B)
        self.stat = self.fbuf("stat", 4)
        self.conf = self.ibuf("conf", 256)

    def fedavg_buffer(self) -> torch.Tensor:
        """Device scratch of numel + 1 floats for the stacked FedAvg (weighted sum | Σw)."""
        buf = getattr(self, "_fedavg_buf", None)
        if buf is None or buf.numel() != self.numel + 1:
            buf = self._fedavg_buf = torch.empty(self.numel + 1, dtype=torch.float32, device=self.device)
        return buf

    def _run_fit_batch(self, batch: Dict[int, tuple]) -> Dict[int, tuple]:
        with self.lock, torch.cuda.device(self.device):
            self._ensure()
            self._common_buffers()
            specs = list(batch.values())
            spec, epochs = specs[0][0], max(r[1] for r in specs)
            extras_any = [r[2] for r in specs if r[2]]
            opt = {
                "kind": 0 if spec.get("name", "sgd") == "adam" else 1, "lr": float(spec.get("lr", 0.01)) * _native.debug_update_scale(),
                "momentum": float(spec.get("momentum", 0.0)),
                "weight_decay": float(spec.get("weight_decay", 0.0)), "nesterov": int(bool(spec.get("nesterov", False))), "mu": 0.0,
            }
            if opt["kind"] == 0:
                raise ValueError("CNN engine implements SGD (the models' optimizer); Adam is not supported here")
            if any("anchor" in e for e in extras_any):
                anchor = self._extra_buffer("anchor")
                opt["mu"] = float(next(e["mu"] for e in extras_any if "anchor" in e))
                for slot, (_, _, extra) in batch.items():
                    anchor[slot, : self.n_params].copy_(extra["anchor"] if "anchor" in extra else self.params[slot, : self.n_params])
                opt["anchor"] = anchor
            if any("c_global" in e for e in extras_any):
                cg, cl = self._extra_buffer("c_global"), self._extra_buffer("c_local")
                for slot, (_, _, extra) in batch.items():
                    if "c_global" in extra:
                        cg[slot, : self.n_params].copy_(extra["c_global"])
                        cl[slot, : self.n_params].copy_(extra["c_local"])
                    else:
                        cg[slot].zero_()
                        cl[slot].zero_()
                opt["cg"], opt["cl"] = cg, cl
            self._opt = opt
            # inactive slots must not train: zero their sample count for this fit
            n_host = [self.n_train[s] if s in batch else 0 for s in range(self.capacity)]
            self._h2d(self.tab["n"], n_host)
            self._fit_seq += 1
            for slot in batch:
                self._slot_fit[slot] = self._fit_seq
            self._h2d(self._fit_id, [self._fit_seq if s in batch else 0 for s in range(self.capacity)])
            self.mom.zero_()
            self._shadow_sync()
            self.stat.zero_()
            steps = (max(n_host) + self.B - 1) // self.B  # host copy: no device round trip
            key = ("fit", steps, tuple(sorted(opt)), opt.get("kind"))
            for ep in range(epochs):
                if self.perm_fn is not None:
                    self.perm.copy_(self.perm_fn(ep))
                else:
                    keys = torch.rand(self.capacity, self.nmax, device=self.device)
                    keys.masked_fill_(self._perm_mask, 2.0)
                    self.perm.copy_(torch.argsort(keys, dim=1).to(torch.int32))
                self._run_steps(key, steps, lambda: [self._train_step(t * self.B) for t in range(steps)], scalars=opt)
            raw = self._d2h_async(self.stat.view(self.capacity, 4))
            self._h2d(self.tab["n"], list(self.n_train))
        # results resolve off-thread when the pinned copy lands (the round never waits for the GPU)
        out = {}
        for slot in batch:
            n = max(1, self.n_train[slot] * epochs)
            out[slot] = (int((self.n_train[slot] + self.B - 1) // self.B) * epochs,
                         raw.map(lambda r, s=slot, n=n: (float(r[0][s, 0]) / n, float(r[0][s, 1]) / n)))
        return out

    def interrupt(self, slot: int) -> None:
        """Stop ``slot``'s running fused fit at the next step (reference: a Lightning fit stopped
        mid-epoch, ``lightning_learner.py:110-114``): its stop word takes the fit's id, and the
        step's input kernel gives that peer an empty batch from then on (no forward, no gradient,
        no optimizer update); the other peers of the gang train on. LeNet-5's one-kernel step and
        a fit already finished are not affected."""
        fid = self._slot_fit.get(slot)
        if fid:
            self._stop[slot] = fid

    def _h2d(self, dst: torch.Tensor, values) -> None:
        """Stream-ordered upload of a small host list (pinned staging; the caching host allocator
        keeps the buffer alive until the copy ran)."""
        src = torch.tensor(values, dtype=dst.dtype, pin_memory=True)
        dst.copy_(src, non_blocking=True)

    def _d2h_async(self, *tensors: torch.Tensor):
        """Pinned device→host copies of ``tensors`` on the current stream and a Pending of their
        numpy views, completed by the resolver thread once the copies landed."""
        if self.resolver is None:
            self.resolver = Resolver(f"cnn-results-{self.device}")
        hosts = [torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for t in tensors]
        for h, t in zip(hosts, tensors):
            h.copy_(t, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))

        def fetch():
            ev.synchronize()
            return [h.numpy() for h in hosts]

        return self.resolver.submit(fetch)

    def _run_steps(self, key, steps: int, body, scalars: Optional[dict] = None) -> None:
        """Run ``body`` (a whole epoch of steps). The first run of a key is eager (it allocates every
        buffer) and is captured into a HIP graph right after it ran; later runs replay the graph.
        Capturing in the first round keeps the capture's host time (the GPU idles through it) out
        of every later round (``MYFYP_CNN_CAPTURE_LATE=1``: capture on the second run instead).
        The graph bakes the optimizer scalars and step offsets in, so they are part of the key."""
        if self.eager or steps == 0:
            body()
            return
        gkey = key + tuple(sorted((k, v) for k, v in (scalars or {}).items() if isinstance(v, (int, float))))
        g = self._graphs.get(gkey)
        if g is None:
            late = os.environ.get("MYFYP_CNN_CAPTURE_LATE", "0") == "1"
            if gkey not in self._seen:
                self._seen.add(gkey)
                body()
                if late:
                    return
                self._graphs[gkey] = self._capture(body)
                return
            g = self._graphs[gkey] = self._capture(body)
        g.replay()

    def _capture(self, body) -> "torch.cuda.CUDAGraph":
        cur = torch.cuda.current_stream(self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(cur)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            body()
        cur.wait_stream(s)
        return g

    def _eval_all(self) -> None:
        steps = (self.ntmax + self.B - 1) // self.B

        def body():
            for t in range(steps):
                if self.arch != "resnet18" and self.lenet_fused:
                    self._lenet_fused(False, t * self.B)
                    continue
                x0 = self._prep(False, t * self.B)
                logits = self._forward_resnet(x0, False) if self.arch == "resnet18" else self._forward_lenet(x0, False)
                self._xent(logits, False)

        self._run_steps(("eval", steps), steps, body)

    def _run_eval_batch(self, batch: Dict[int, tuple]) -> Dict[int, tuple]:
        with self.lock, torch.cuda.device(self.device):
            self._ensure()
            self._common_buffers()
            self._shadow_sync()
            self.stat.zero_()
            self.conf.zero_()
            self._eval_all()
            raw = self._d2h_async(self.stat.view(self.capacity, 4), self.conf.view(self.capacity, 16, 16))
        K = self.n_classes
        return {slot: raw.map(lambda r, s=slot: (float(r[0][s, 0]) / max(1, self.n_test[s]), r[1][s, :K, :K].copy())) for slot in batch}

    def expect(self, fit_slots: Optional[Set[int]] = None, eval_slots: Optional[Set[int]] = None) -> None:
        self.fit_gang.expected = fit_slots
        self.eval_gang.expected = eval_slots

    def default_expected(self) -> Set[int]:
        return set(self.handles)


class CNNEngineHandle:
    """A learner's slot in a :class:`CNNGroup` (same interface as ``MLPEngineHandle``)."""

    @staticmethod
    def supports(module: torch.nn.Module) -> bool:
        if arch_of(module) is None:
            return False
        if _native.load() is None:
            raise RuntimeError(f"MI355X CNN engine requested but native library unavailable: {_native.error()}")
        return True

    @classmethod
    def attach(cls, module: torch.nn.Module, device: torch.device, addr: str, learner=None, batch_size: Optional[int] = None, tag=None) -> "CNNEngineHandle":
        return cls(module, device, addr, int(batch_size or Settings.BATCH_SIZE), learner, tag)

    def __init__(self, module: torch.nn.Module, device: torch.device, addr: str, batch_size: int, learner=None, tag=None) -> None:
        self.addr, self.module, self.learner = addr, module, learner
        self.group = CNNGroup.get(device, module, batch_size, tag)
        self._data_id = id(learner.data) if learner is not None else None
        with self.group.lock:
            self.slot = self.group.attach(self)
            self.retarget(copy_in=True)

    def retarget(self, copy_in: bool = False) -> None:
        g = self.group
        row = g.params[self.slot]
        with torch.no_grad():
            off = 0
            for p in self.module.parameters():
                view = row[off : off + p.numel()].view_as(p)
                if copy_in:
                    view.copy_(p.data.to(view.dtype))
                p.data = view
                off += p.numel()
            for bn in g.bns:
                mod = self._module_bn(bn.name)
                o = g.n_params + g.bn_off[bn.name]
                rm = row[o : o + bn.C]
                rv = row[o + g.bn_total : o + g.bn_total + bn.C]
                if copy_in:
                    rm.copy_(mod.running_mean.float())
                    rv.copy_(mod.running_var.float())
                mod.running_mean = rm
                mod.running_var = rv

    def _module_bn(self, name: str):
        import re

        m = self.module
        if name == "stem_bn":
            return m.bn1
        mt = re.fullmatch(r"b(\d+)(bn1|bn2|sbn)", name)
        blk = m.layers[int(mt.group(1))]
        return {"bn1": blk.bn1, "bn2": blk.bn2, "sbn": blk.shortcut[1] if len(blk.shortcut) else None}[mt.group(2)]

    def close(self) -> None:
        self.group.detach(self.slot)

    def interrupt(self) -> None:
        """Stop this peer's running fused fit at the next step (``CNNGroup.interrupt``)."""
        self.group.interrupt(self.slot)

    def flat_params(self) -> torch.Tensor:
        return self.group.params[self.slot, : self.group.n_params]

    def device_split(self, train: bool) -> Tuple[torch.Tensor, torch.Tensor]:
        g = self.group
        if self.learner is None or self.learner.data is None:
            return torch.zeros(0, g.in_h, g.in_w, g.in_c, dtype=torch.uint8, device=g.device), torch.zeros(0, dtype=torch.int64, device=g.device)
        x, y = self.learner.device_data(train)
        if x.dtype != torch.uint8:
            raise TypeError("CNN engine expects uint8 images")
        x = x.reshape(x.shape[0], g.in_h, g.in_w, g.in_c).contiguous()
        return x, y.to(torch.int64).contiguous()

    def _sync_data(self, learner) -> None:
        if self.learner is not learner or self._data_id != id(learner.data):
            self.learner = learner
            self._data_id = id(learner.data)
            self.group.invalidate_data()

    def fit(self, learner, spec: dict, extra: dict) -> Tuple[int, float]:
        self._sync_data(learner)
        steps, raw = self.group.fit_gang.submit(self.slot, (spec, learner.epochs, extra), self.group.default_expected())
        learner.global_step += steps
        return steps, raw.map(lambda v: v[0])

    def evaluate(self, learner) -> Tuple[float, np.ndarray]:
        self._sync_data(learner)
        return self.group.eval_gang.submit(self.slot, (), self.group.default_expected())
