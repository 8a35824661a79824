"""Phase timing inside the tile-split backward from s_memtime stamps (diagnostic build).

    make -C insr-pde_amd/csrc diag && python tools/diag_stamps.py [--net fluid_pres] [--mode lap] [--n 16384]

Phases per layer j (L..1): 0->1 sine reverse + bias partials, 1->2 sin/cos of z_{j-1}
(global loads), 2->3 barrier 1, 3->4 LDS writes (zb, h_{j-1}), 4->5 barrier 2,
5->6 dW MFMAs + stores, 6->7 propagation (W^T loads + MFMAs).  Cycles, median over
the waves of block 0 and of the middle block.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
import torch  # noqa: E402

NETS = {"fluid_pres": (2, 1, 4, 128), "fluid_vel": (2, 2, 4, 128), "el3d": (3, 3, 5, 256)}
PH = ["sine_rev+bias", "sincos(z_j-1)", "barrier1", "lds_write", "barrier2", "dW", "propagate"]
# x6 backward (jet_x6.hpp): stamps of the LAST stream group of a layer
PH_X6 = ["sine_rev+bias", "W^T frags+sincos(+prev groups)", "barrier1", "lds_write", "barrier2", "dW", "propagate"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--net", default="fluid_pres")
    ap.add_argument("--mode", default="lap")
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--prec", type=int, default=0, help="1: split-bf16 (x6) kernels")
    ap.add_argument("--fprec", type=int, default=None, help="INSR_PREC_* of the forward (with --bprec)")
    ap.add_argument("--bprec", type=int, default=None, help="INSR_PREC_* of the backward; with the default "
                    "f16 mask a bf16x6 backward runs the fused kernel on fp16 products (f16x3)")
    args = ap.parse_args()
    import base
    from base import _native as nat
    lib = nat.load(os.path.join(ROOT, "insr-pde_amd", "lib", "libinsr_hip_diag.so"))
    lib.insr_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.insr_diag_stamps_x6.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.insr_diag_stamps_h.argtypes = [ctypes.c_void_p, ctypes.c_int]
    f16 = args.bprec is not None
    prec = (args.fprec, args.bprec) if f16 else (args.prec, args.prec)
    ph = PH_X6 if (args.prec or f16) else PH
    din, dout, L, W = NETS[args.net]
    mode = {"value": 0, "grad": 1, "lap": 2}[args.mode] | nat.knob_bits(prec=prec)
    n = args.n
    torch.manual_seed(0)
    net = base.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    flat = net.flat_params()
    x = (torch.rand(n, din, device="cuda") * 2 - 1).contiguous()
    y, dy, lap = (torch.empty(n, dout, device="cuda"), torch.empty(n, dout, din, device="cuda"),
                  torch.empty(n, dout, device="cuda"))
    gy, gdy, glap = torch.randn_like(y), torch.randn_like(dy), torch.randn_like(lap)
    act = torch.empty(lib.insr_jet_act_bytes(n, din, L, W, mode) // 4, device="cuda")
    part = torch.empty(lib.insr_jet_partial_bytes(n, din, dout, L, W, mode) // 4, device="cuda")
    st = nat.stream_of(x.device)
    nat.check(lib.insr_siren_jet_fwd(nat.ptr(x), n, din, dout, L, W, mode, nat.ptr(flat), nat.ptr(y), nat.ptr(dy),
                                     nat.ptr(lap), nat.ptr(act), st), "fwd")
    for _ in range(3):
        nat.check(lib.insr_siren_jet_bwd(nat.ptr(x), n, din, dout, L, W, mode, nat.ptr(flat), nat.ptr(act),
                                         nat.ptr(gy), nat.ptr(gdy), nat.ptr(glap), nat.ptr(part), st), "bwd")
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (2 * 16 * 8 * 8))()
    (lib.insr_diag_stamps_h if f16 else lib.insr_diag_stamps_x6 if args.prec else lib.insr_diag_stamps)(buf, len(buf))
    T = lib.insr_jet_split_tiles(n, din, W, mode, 1)
    print(f"{args.net} {args.mode} n={n} T={T} prec={prec}")
    for blk in (0, 1):
        rows = []
        for wave in range(8):
            for layer in range(L):  # hidden layers j = L..1 (slot 0..L-1)
                b = ((blk * 16 + wave) * 8 + layer) * 8
                v = [buf[b + k] for k in range(8)]
                if v[0] and v[7]:
                    rows.append([v[k + 1] - v[k] if k != 1 else v[2] - v[1] for k in range(7)])
        if not rows:
            continue
        med = [sorted(r[k] for r in rows)[len(rows) // 2] for k in range(7)]
        tot = sum(med)
        print(f" block {'0' if blk == 0 else 'mid'}: layer total {tot} cyc; " +
              ", ".join(f"{ph[k]} {med[k]} ({100 * med[k] / max(tot, 1):.0f}%)" for k in range(7)))


if __name__ == "__main__":
    main()
