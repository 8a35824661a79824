"""Kernel micro-benchmark: fwd / bwd jet kernels back-to-back on one stream
(HIP events around R launches, no host gaps), for both kernel variants.

    python tools/kbench.py [--nets fluid_pres,fluid_vel] [--sizes 324,4096,16384]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

import torch  # noqa: E402

NETS = {"fluid_pres": (2, 1, 4, 128), "fluid_vel": (2, 2, 4, 128), "advect": (1, 1, 3, 64),
        "el2d": (2, 2, 5, 128), "el3d": (3, 3, 5, 256)}
VARIANTS = {  # label: ((fwd, bwd) forced tiles, (fwd, bwd) precision)
    "split1": ((1, 1), (0, 0)),
    "split2": ((2, 2), (0, 0)),
    "split4": ((4, 4), (0, 0)),
    "auto": ((0, 0), (0, 0)),
    "x6": ((0, 0), (1, 1)),
    "x6_1": ((1, 1), (1, 1)),
    "x6_2": ((2, 2), (1, 1)),
    "x6_4": ((4, 4), (1, 1)),
    "x6w": ((0, 0), (1, 1)),  # x6 with the two-kernel backward from width 128
    "x3": ((0, 0), (2, 2)),   # 3 bf16 products per fp32 product
    "bf": ((0, 0), (3, 3)),   # plain bf16 operands
    "h3": ((0, 0), (4, 1)),   # fp16 two-term forward (f16x3), x6 backward
}
MODES = {"value": 0, "grad": 1, "lap": 2}


def P_macs(din, dout, L, W):
    return din * W + L * W * W + W * dout


def time_it(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nets", default="fluid_pres,fluid_vel")
    ap.add_argument("--sizes", default="324,2048,8192,16384,65536")
    ap.add_argument("--modes", default="value,grad,lap")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--policies", default="0", help="backward-path policies (INSR_JET_POLICY mode bits) to time")
    ap.add_argument("--bwd-only", action="store_true", help="time only the backward into .grad")
    ap.add_argument("--bwd-f16", type=int, default=-1, help="INSR_JET_BWD_F16 mask (-1: library default)")
    ap.add_argument("--lib", default=None, help="alternative build of libinsr_hip.so (flag studies)")
    args = ap.parse_args()
    import base
    from base import _native as nat
    lib = nat.load(args.lib, check_build=args.lib is None)
    f16bits = nat.jet_bwd_f16(args.bwd_f16) if args.bwd_f16 >= 0 else 0
    out = []
    for name in args.nets.split(","):
        din, dout, L, W = NETS[name]
        torch.manual_seed(0)
        net = base.MLP(din, dout, L, W, nonlinearity="sine").cuda()
        flat = net.flat_params()
        try:  # libraries with pre-split weight planes: prepare them once, pass INSR_MODE_WSPLIT
            lib.insr_siren_wsplit
            net.refresh_wsplit()
            wbit = nat.MODE_WSPLIT
        except AttributeError:
            wbit = 0
        P = net.param_count
        for mname in args.modes.split(","):
            mode0 = MODES[mname] | wbit | f16bits
            if (mode0 & 0xF) == 2 and din > 2:
                continue
            S = {0: 1, 1: 1 + din, 2: 2 + din}[mode0 & 0xF]
            for n in [int(v) for v in args.sizes.split(",")]:
                x = (torch.rand(n, din, device="cuda") * 2 - 1).contiguous()
                y = torch.empty(n, dout, device="cuda")
                dy = torch.empty(n, dout, din, device="cuda")
                lap = torch.empty(n, dout, device="cuda")
                gy, gdy, glap = torch.randn_like(y), torch.randn_like(dy), torch.randn_like(lap)
                act = torch.empty(lib.insr_jet_act_bytes(n, din, L, W, mode0) // 4, device="cuda")
                g = torch.zeros(P, device="cuda")
                st = nat.stream_of(x.device)
                for variant, pol in [(v, int(p)) for v in args.variants.split(",") for p in args.policies.split(",")]:
                    tiles, prec = VARIANTS[variant]
                    # the variant as per-call mode bits (the library keeps no configuration)
                    mode = mode0 | nat.knob_bits(policy=pol, tiles=tiles, prec=prec, wide128=variant.endswith("w"))
                    part = torch.empty(max(lib.insr_jet_partial_bytes(n, din, dout, L, W, mode) // 4, 1), device="cuda")
                    nb = lib.insr_jet_partial_blocks(n, din, W, mode)
                    tf_, tb_ = (lib.insr_jet_split_tiles(n, din, W, mode, 0),
                                lib.insr_jet_split_tiles(n, din, W, mode, 1))

                    def fwd():
                        nat.check(lib.insr_siren_jet_fwd(nat.ptr(x), n, din, dout, L, W, mode, nat.ptr(flat),
                                                         nat.ptr(y), nat.ptr(dy), nat.ptr(lap), nat.ptr(act), st),
                                  "fwd")

                    def bwd():
                        nat.check(lib.insr_siren_jet_bwd(nat.ptr(x), n, din, dout, L, W, mode, nat.ptr(flat),
                                                         nat.ptr(act), nat.ptr(gy), nat.ptr(gdy), nat.ptr(glap),
                                                         nat.ptr(part), st), "bwd")

                    work = torch.empty(max(lib.insr_jet_bwd_work_bytes(n, din, dout, L, W, mode) // 4, 1),
                                       device="cuda")
                    wide = lib.insr_jet_bwd_is_wide(n, din, W, mode)

                    def bwdg():  # backward straight into .grad (the path the autograd bridge takes)
                        nat.check(lib.insr_siren_jet_bwd_grad(nat.ptr(x), n, din, dout, L, W, mode, nat.ptr(flat),
                                                              nat.ptr(act), nat.ptr(gy), nat.ptr(gdy), nat.ptr(glap),
                                                              nat.ptr(work), nat.ptr(g), 0, st), "bwd_grad")

                    def red():
                        nat.check(lib.insr_reduce_partials_strided(nat.ptr(part), nb, P,
                                                                   lib.insr_jet_partial_stride(din, dout, L, W),
                                                                   nat.ptr(g), 0, st), "reduce")

                    tf = time_it(fwd, args.reps)
                    fwd()
                    tb = 1e9 if args.bwd_only else time_it(bwd, args.reps)
                    tr = 1e9 if args.bwd_only else time_it(red, args.reps)
                    tg = time_it(bwdg, args.reps)
                    macs = P_macs(din, dout, L, W)
                    rec = {"net": name, "mode": mname, "n": n, "variant": variant, "policy": pol,
                           "path": lib.insr_jet_bwd_path(n, din, dout, L, W, mode), "T": [tf_, tb_], "nb": nb,
                           "fwd_us": round(tf, 2),
                           "bwd_us": round(tb, 2), "reduce_us": round(tr, 2), "bwd_grad_us": round(tg, 2),
                           "wide": wide, "bwd_grad_tflops": round(n * S * 4 * macs / tg / 1e6, 2),
                           "fwd_tflops": round(n * S * 2 * macs / tf / 1e6, 2),
                           "bwd_tflops": round(n * S * 4 * macs / tb / 1e6, 2)}
                    out.append(rec)
                    print(json.dumps(rec), flush=True)



if __name__ == "__main__":
    main()
