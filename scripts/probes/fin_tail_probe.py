"""Cost of the fused BatchNorm finalize tail (conv.hip conv_fin_tail) on forward convs of the
ResNet-18 config-4 shapes (8 peers x batch 128): the same launch without the tail, with it, and
with parts of it switched off through conv_set_fin_debug (timing only: 1 = no vmcnt wait, 2 = no
arrival ticket, 4 = ticket but no finalize work). GPU only."""
import ctypes
import json
import sys

import torch

from myfyp_amd.parallel.cnn_engine import ConvGemmArgs, _lib


def main() -> None:
    lib = _lib()
    dev = torch.device("cuda")
    P, B = 8, 128
    s = torch.cuda.current_stream().cuda_stream
    nb = torch.full((P,), B, dtype=torch.int32, device=dev)
    out = []
    for (h, c, stride) in [(32, 64, 1), (16, 128, 1), (8, 256, 1), (4, 512, 1)]:
        ho = h
        x = (torch.randn(P, B * h * h * c, device=dev)).to(torch.bfloat16)
        wf = (torch.randn(P, c * 9 * c, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(P, B * ho * ho * c, dtype=torch.bfloat16, device=dev)
        rows = lib.conv_gemm_stats_rows(B, ho, ho)
        stats = torch.zeros(P, rows * 2 * c, device=dev)
        cnt = torch.zeros(P, lib.conv_fin_words(), dtype=torch.int32, device=dev)
        prm = torch.ones(P, 4 * c, device=dev)
        ss, ms = torch.zeros(P, 2 * c, device=dev), torch.zeros(P, 2 * c, device=dev)
        a = ConvGemmArgs()
        a.src, a.src_ps, a.src_h, a.src_w, a.src_c = x.data_ptr(), x.shape[1], h, h, c
        a.out_h, a.out_w, a.R, a.S, a.stride, a.pad = ho, ho, 3, 3, stride, 1
        a.wt, a.wt_ps, a.ncol, a.ncol_valid = wf.data_ptr(), wf.shape[1], c, c
        a.out, a.out_ps, a.stats, a.stats_ps, a.stats_rows = y.data_ptr(), y.shape[1], stats.data_ptr(), stats.shape[1], rows
        a.nbatch, a.max_batch = nb.data_ptr(), B
        row = {"h": h, "c": c}

        def timed(tag):
            for _ in range(3):
                assert lib.conv_gemm_launch(0, ctypes.byref(a), P, s) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                lib.conv_gemm_launch(0, ctypes.byref(a), P, s)
            e1.record()
            torch.cuda.synchronize()
            row[tag] = round(e0.elapsed_time(e1) * 1000 / 20, 2)

        timed("no_tail")
        stats.zero_()
        a.fin_cnt, a.fin_gamma0, a.fin_beta, a.fin_param_ps = cnt.data_ptr(), prm.data_ptr(), prm.data_ptr() + 4 * c, prm.shape[1]
        a.fin_rmean, a.fin_rvar, a.fin_run_ps = prm.data_ptr() + 8 * c, prm.data_ptr() + 12 * c, prm.shape[1]
        a.fin_ss, a.fin_ms, a.fin_C0, a.fin_train, a.fin_eps, a.fin_momentum = ss.data_ptr(), ms.data_ptr(), c, 1, 1e-5, 0.1
        for dbg in (0, 1, 2, 4):
            lib.conv_set_fin_debug(dbg)
            cnt.zero_()
            stats.zero_()
            timed(f"tail_dbg{dbg}")
        lib.conv_set_fin_debug(0)
        a.fin_train = 0
        cnt.zero_()
        timed("tail_eval")
        a.fin_cnt = None
        a.stats = None
        timed("no_stats_no_tail")
        print(json.dumps(row), flush=True)
        out.append(row)
    json.dump(out, open(sys.argv[1], "w") if len(sys.argv) > 1 else sys.stdout, indent=1)


if __name__ == "__main__":
    main()
