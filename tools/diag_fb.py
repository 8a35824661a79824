"""Phase timing inside the recompute backward (jet_fb.hpp) from s_memtime stamps (diagnostic build).

    make -C insr-pde_amd/csrc diag && python tools/diag_fb.py [--n 16708] [--net fluid_pres]

Stamps per tile (block 0, every wave, first 8 tiles): the forward's layer 0 + its planes, per hidden
layer the MFMAs and the planes of the next, the output-layer reverse, per reverse layer the sine
reverse, the block-maximum exchange (barrier), the P / H writes (+ barrier), the dW MFMAs, the
propagation; cycles (s_memtime ticks), median over the waves and tiles.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]
import torch  # noqa: E402

NETS = {"fluid_pres": (2, 1, 4, 128, 2), "fluid_vel": (2, 2, 4, 128, 0)}


def phases(L, saved=False):
    if saved:  # the saved-stream variant (policy 5): no forward, the output layer reads z_L
        names = [(0, 10, "out-layer rev (+ z_L load)")]
        prev = 10
        for j in range(L, 0, -1):
            sp = 11 + 5 * (L - j)
            names += [(prev, sp, f"rev L{j} sine_rev+z"), (sp, sp + 1, f"rev L{j} exchange"),
                      (sp + 1, sp + 2, f"rev L{j} P/H writes"), (sp + 2, sp + 3, f"rev L{j} dW"),
                      (sp + 3, sp + 4, f"rev L{j} prop")]
            prev = sp + 4
        names.append((prev, 31, "rev L0"))
        return names
    names = [(0, 1, "fwd L0 + planes")]
    for j in range(1, L + 1):
        names.append((2 * j - 1, 2 * j, f"fwd L{j} MFMA"))
        names.append((2 * j, 2 * j + 1, f"fwd L{j} planes" if j < L else f"fwd L{j} save"))
    names.append((2 * L + 1, 10, "out-layer rev"))
    prev = 10
    for j in range(L, 0, -1):
        sp = 11 + 5 * (L - j)
        names += [(prev, sp, f"rev L{j} sine_rev+z"), (sp, sp + 1, f"rev L{j} exchange"),
                  (sp + 1, sp + 2, f"rev L{j} P/H writes"), (sp + 2, sp + 3, f"rev L{j} dW"),
                  (sp + 3, sp + 4, f"rev L{j} prop")]
        prev = sp + 4
    names.append((prev, 31, "rev L0"))
    return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--net", default="fluid_pres")
    ap.add_argument("--n", type=int, default=16708)
    ap.add_argument("--policy", type=int, default=4, choices=[4, 5], help="4 recompute, 5 saved-stream variant")
    args = ap.parse_args()
    import base
    from base import _native as nat
    lib = nat.load(os.path.join(ROOT, "insr-pde_amd", "lib", "libinsr_hip_diag.so"), check_build=False)
    lib.insr_diag_fb_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    din, dout, L, W, mode = NETS[args.net]
    n = args.n
    torch.manual_seed(0)
    net = base.MLP(din, dout, L, W, nonlinearity="sine").cuda()
    net.refresh_wsplit()
    flat = net.flat_params()
    cm = mode | nat.MODE_WSPLIT | nat.jet_policy(args.policy)
    assert lib.insr_jet_bwd_path(n, din, dout, L, W, cm) == (3 if args.policy == 4 else 2)
    x = (torch.rand(n, din, device="cuda") * 2 - 1).contiguous()
    act = None
    if args.policy == 5:  # the forward's saved streams
        act = torch.empty(lib.insr_jet_act_bytes(n, din, L, W, cm) // 4, device="cuda")
        y, dy, lp = (torch.empty(n, dout, device="cuda"), torch.empty(n, dout, din, device="cuda"),
                     torch.empty(n, dout, device="cuda"))
        nat.check(lib.insr_siren_jet_fwd(nat.ptr(x), n, din, dout, L, W, cm, nat.ptr(flat), nat.ptr(y), nat.ptr(dy),
                                         nat.ptr(lp), nat.ptr(act), nat.stream_of(x.device)), "fwd")
    gy = torch.randn(n, dout, device="cuda")
    gdy = torch.randn(n, dout, din, device="cuda") if mode else None
    glap = torch.randn(n, dout, device="cuda") if mode == 2 else None
    work = torch.empty(lib.insr_jet_bwd_work_bytes(n, din, dout, L, W, cm) // 4, device="cuda")
    grad = torch.zeros(net.param_count, device="cuda")
    st = nat.stream_of(x.device)
    for _ in range(3):
        nat.check(lib.insr_siren_jet_bwd_grad(nat.ptr(x), n, din, dout, L, W, cm, nat.ptr(flat), nat.ptr(act), nat.ptr(gy),
                                              nat.ptr(gdy), nat.ptr(glap), nat.ptr(work), nat.ptr(grad), 0, st), "bwd")
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (8 * 8 * 32))()
    nat.check(lib.insr_diag_fb_stamps(buf, len(buf)), "stamps")
    ph = phases(L, args.policy == 5)
    rows = []
    for wave in range(8):
        for t in range(8):
            b = (wave * 8 + t) * 32
            v = [buf[b + k] for k in range(32)]
            if v[0] and v[31] and v[31] > v[0]:
                rows.append([v[e] - v[s] for s, e, _ in ph] + [v[31] - v[0]])
    print(f"{args.net} n={n}: {len(rows)} (wave, tile) samples")
    if not rows:
        return
    med = [sorted(r[k] for r in rows)[len(rows) // 2] for k in range(len(ph) + 1)]
    tot = med[-1]
    print(f"tile total {tot} cycles (median)")
    for (s, e, name), m in zip(ph, med):
        print(f"  {name:22s} {m:7d}  {100.0 * m / tot:5.1f}%")


if __name__ == "__main__":
    main()
