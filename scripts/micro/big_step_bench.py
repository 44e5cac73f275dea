"""Per-time-step cost of the large-H LSTM step (H = 2048, BASELINE config 4): the fused MFMA step
kernels (csrc/lstm_gemm_step.hip) vs the library form (hipBLASLt GEMM + epilogue-only cell kernel,
csrc/lstm_ew.hip).  Each variant runs 32 back-to-back steps captured in a hipGraph; us per step.

  python scripts/micro/big_step_bench.py [--H 2048] [--B 64,256,1024] [--S 0]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_char_rnn_amd.ops import native  # noqa: E402

NSTEP = 32


def graph_time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / NSTEP)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=2048)
    ap.add_argument("--B", default="64,128,256,512,1024")
    ap.add_argument("--S", type=int, default=0)
    ap.add_argument("--cfgs", default="", help="tile configuration ids to time (bigstep_cfg)")
    a = ap.parse_args()
    ops = native.ops()
    H = a.H
    dev = "cuda"
    WhT = (torch.randn(4 * H, H, device=dev) / H ** 0.5).to(torch.bfloat16)
    Wh = WhT.t().contiguous()
    for B in (int(x) for x in a.B.replace(":", ",").split(",")):
        h = torch.randn(NSTEP + 1, B, H, device=dev).to(torch.bfloat16)
        c = torch.randn(NSTEP + 1, B, H, device=dev)
        zx = torch.randn(B, 4 * H, device=dev)
        gates = torch.rand(NSTEP, B, 4 * H, device=dev).to(torch.bfloat16)
        dz = torch.randn(NSTEP + 1, B, 4 * H, device=dev).to(torch.bfloat16)
        dtop = torch.randn(B, H, device=dev)
        dc = torch.zeros(B, H, device=dev)
        zrec = torch.empty(1, B, 4 * H, device=dev)
        wf, nt = ops.big_step_workspace(False, B, H, a.S)
        wsf = torch.empty(max(wf, 4), device=dev)
        cf = torch.zeros(max(nt, 1), dtype=torch.int32, device=dev)
        wb, ntb = ops.big_step_workspace(True, B, H, a.S)
        wsb = torch.empty(max(wb, 4), device=dev)
        cb = torch.zeros(max(ntb, 1), dtype=torch.int32, device=dev)
        S = 4 if B >= 512 else 2 if B >= 256 else 1
        dh = torch.empty(S, B, H, device=dev)
        WhTs = Wh.t() if S == 1 else Wh.view(H, S, 4 * H // S).permute(1, 2, 0)

        def fused_fwd():
            for t in range(NSTEP):
                ops.lstm_big_step_fwd(WhT, h[t], zx, None, c[t], h[t + 1], None, c[t + 1],
                                      gates[t], wsf, cf, 1.0, a.S)

        def lib_fwd():
            for t in range(NSTEP):
                torch.mm(h[t], WhT.t(), out_dtype=torch.float32, out=zrec[0])
                ops.lstm_step_ew_fwd(zrec, zx, None, c[t], h[t + 1], None, c[t + 1], gates[t], 1.0)

        def fused_bwd():
            for t in range(NSTEP):
                ops.lstm_big_step_bwd(Wh, dz[t + 1], dtop, gates[t], c[t + 1], c[t], dc, dz[t],
                                      wsb, cb, a.S)

        def lib_bwd():
            for t in range(NSTEP):
                if S == 1:
                    torch.mm(dz[t + 1], WhTs, out_dtype=torch.float32, out=dh[0])
                else:
                    torch.bmm(dz[t + 1].view(B, S, 4 * H // S).transpose(0, 1), WhTs,
                              out_dtype=torch.float32, out=dh)
                ops.lstm_step_ew_bwd(dtop, dh, gates[t], c[t + 1], c[t], dc, dz[t])

        fl = 2.0 * B * 4 * H * H
        if a.cfgs:
            for cid in (int(x) for x in a.cfgs.replace(":", ",").split(",")):
                os.environ["DCR_DEBUG"] = f"bigstep_cfg={cid}"
                bwd = cid in (2, 3, 5) or cid >= 8
                # the workspace depends on the configuration's tile count
                wf, nt = ops.big_step_workspace(bwd, B, H, a.S)
                ws_c = torch.empty(max(wf, 4), device=dev)
                cnt_c = torch.zeros(max(nt, 1), dtype=torch.int32, device=dev)
                if bwd:
                    wsb, cb = ws_c, cnt_c
                else:
                    wsf, cf = ws_c, cnt_c
                t = graph_time(fused_bwd if bwd else fused_fwd)
                print(f"H={H} B={B:5d}  cfg {cid} ({'bwd' if bwd else 'fwd'}) {t:7.2f} us "
                      f"({fl / t / 1e6:6.1f} TF/s)", flush=True)
            os.environ.pop("DCR_DEBUG", None)
            continue
        tf, tl = graph_time(fused_fwd), graph_time(lib_fwd)
        bf, bl = graph_time(fused_bwd), graph_time(lib_bwd)
        print(f"H={H} B={B:5d}  fwd fused {tf:7.2f} us ({fl / tf / 1e6:6.1f} TF/s)  library {tl:7.2f} us"
              f"  |  bwd fused {bf:7.2f} us ({fl / bf / 1e6:6.1f} TF/s)  library {bl:7.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
