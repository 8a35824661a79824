"""C ABI checks that need no GPU: the library loads, exports every symbol that
include/insr_siren.h declares, and the pure-host queries answer correctly."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "insr_siren.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|long|void|const char\*)\s+(insr_\w+)\s*\(", txt, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as ge
    ge.build()
    import base
    return base._native.load(ge.LIB)


def test_header_matches_binding():
    from base import _native as nat
    assert declared_symbols() == sorted(nat.SIGNATURES)


def test_header_constants_match_binding():
    """The optimiser-state layout and mode-bit constants the Python side allocates / passes are the
    header's (#define NAME value, integers only)."""
    import re
    from base import _native as nat
    text = open(HEADER).read()
    defs = dict(re.findall(r"#define (INSR_OPT_\w+) (\d+)\b", text))
    for name, value in defs.items():
        assert getattr(nat, name[len("INSR_"):]) == int(value), name
    assert "INSR_OPT_NFLOATS" in defs and "INSR_OPT_TICKET_SHARDS" in defs


def test_exports_every_declared_symbol(lib):
    import ctypes
    for name in declared_symbols():
        assert isinstance(getattr(lib, name), ctypes._CFuncPtr), name


def test_build_id_matches_sources(lib):
    """The loaded library was built from the checked-out csrc/ + header (load() enforces it)."""
    from base import _native as nat
    assert lib.insr_build_id().decode() == nat.source_hash()


def test_host_queries(lib):
    assert lib.insr_version() >= 100
    # SURVEY.md §8 parameter counts, verified against the reference MLP
    assert lib.insr_siren_param_count(1, 1, 3, 64) == 12673
    assert lib.insr_siren_param_count(2, 2, 4, 128) == 66690
    assert lib.insr_siren_param_count(2, 1, 4, 128) == 66561
    assert lib.insr_siren_param_count(2, 2, 5, 128) == 83202
    assert lib.insr_siren_param_count(3, 3, 5, 256) == 330755
    assert lib.insr_siren_supported(2, 1, 4, 128, 2) == 1
    assert lib.insr_siren_supported(3, 1, 4, 128, 2) == 1   # 5-stream Laplacian jet (d_in = 3)
    assert lib.insr_siren_supported(4, 1, 4, 128, 2) == 0   # d_in <= 3
    assert lib.insr_siren_supported(2, 1, 4, 100, 0) == 0   # width not compiled
    # saved activations: (L+1) layers x 16 W floats per 16-point tile x S streams
    assert lib.insr_jet_act_bytes(64, 2, 4, 128, 2) == 5 * 4 * 16 * 128 * 4 * 4
    from base import _native as nat
    assert lib.insr_jet_partial_stride(2, 1, 4, 128) == 66564 and lib.insr_jet_partial_stride(2, 2, 4, 128) == 66692
    assert lib.insr_jet_partial_blocks(0, 2, 128, 2) == 0
    k = nat.jet_tiles(0, 0, 512)                            # per-call knob: auto T, >= 512 blocks
    assert lib.insr_jet_partial_blocks(65, 2, 128, 2 | k) == 5            # small: T = 1
    assert lib.insr_jet_partial_bytes(65, 2, 1, 4, 128, 2 | k) == 5 * 66564 * 4  # rows padded to 4 floats
    assert lib.insr_jet_split_tiles(65, 3, 256, 1 | k, 1) == 1
    # LAP (S=4) at W=128: 70 KB of LDS per tile -> T <= 2; 16384 points = 1024 tiles
    assert lib.insr_jet_split_tiles(16384, 2, 128, 2 | k, 1) == 2
    assert lib.insr_jet_partial_blocks(16384, 2, 128, 2 | k) == 512
    assert lib.insr_jet_split_tiles(16384, 2, 128, 0 | k, 1) == 2         # T=4 would leave 256 blocks
    k = nat.jet_tiles(1, 4, 512)                            # forced: fwd 1, bwd 4 (capped by LDS)
    assert lib.insr_jet_split_tiles(65536, 2, 128, 0 | k, 0) == 1
    assert lib.insr_jet_split_tiles(65536, 2, 128, 2 | k, 1) == 2
    assert lib.insr_jet_partial_blocks(65536, 2, 128, 2 | k) == 2048
    # the knobs live in the call, not in the library: a call without them is unaffected
    assert lib.insr_jet_partial_blocks(16384, 2, 128, 2) == lib.insr_jet_partial_blocks(16384, 2, 128, 2 | nat.jet_tiles())


def test_invalid_arguments_rejected_without_launch(lib):
    # bad shapes are refused before anything touches the device
    assert lib.insr_siren_jet_fwd(None, 10, 0, 1, 4, 128, 0, None, None, None, None, None, None) == -1
    assert lib.insr_siren_jet_fwd(None, 10, 2, 1, 4, 100, 0, None, None, None, None, None, None) == -1
    assert lib.insr_siren_jet_fwd(None, 0, 2, 1, 4, 128, 0, None, None, None, None, None, None) == 0
    assert lib.insr_adam_step(None, None, None, None, 10, None, 0.9, 0.999, 1e-8, None) == -1


def test_comm_library_resolves(lib):
    # RCCL ships with the ROCm image (and with PyTorch-ROCm): the C-ABI collective can load it
    assert lib.insr_comm_available() == 1
    assert lib.insr_comm_id_bytes() == 128
    assert lib.insr_comm_init(None, 0, 1, None) == -1  # INSR_EINVAL, no RCCL call made


def test_struct_layouts_match_header(tmp_path):
    """The ctypes mirrors of the header's structs have the C compiler's size and field offsets."""
    import ctypes
    import subprocess
    from base import _native as nat
    structs = {"InsrJetJob": nat.JetJob, "InsrBwdJob": nat.BwdJob, "InsrLoss": nat.Loss, "InsrBox": nat.Box, "InsrElastic": nat.Elastic}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'  printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                                text=True).stdout.splitlines())
    for cname, py in structs.items():
        assert int(got[f"{cname} size"]) == ctypes.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f"{cname} {fname}"]) == getattr(py, fname).offset, (cname, fname)


def test_mixed_launch_rejects_malformed_jobs(lib):
    """insr_siren_jet_fwd_mixed validates every field jet_fwd_x6_mixed indexes with on the host
    (capi.hip mixed_jobs_ok): a malformed job returns INSR_EINVAL before any device call, so
    these run without a GPU.  Pointers are dummies that are never dereferenced."""
    import ctypes
    from base import _native as nat
    P = [0x10000 * (i + 1) for i in range(12)]  # distinct fake device addresses

    def job(x=P[0], prm=P[1], y=P[2], dy=P[3], lap=P[4], n=64, d_out=0):
        return nat.JetJob(x, prm, y, dy, lap, None, n, d_out)

    def call(jobs, modes, scalars=(0.05, -1.0, 1.0) * 4, din=2, dout=2, prec=0):
        arr = (nat.JetJob * len(jobs))(*jobs)
        md = (ctypes.c_int * len(modes))(*modes)
        sc = None if scalars is None else (ctypes.c_float * len(scalars))(*scalars)
        return lib.insr_siren_jet_fwd_mixed(arr, md, sc, len(jobs), din, dout, 4, 128, prec, None)

    V, G, LAP, ADV = nat.MODE_VALUE, nat.MODE_GRAD, nat.MODE_LAP, 3
    bad = [
        ([job()], [5]),                                   # unknown job mode
        ([job()], [-1]),
        ([job()], [V | 0x10]),                            # precision bits in a job mode
        ([job(d_out=4)], [V]),                            # output width out of range
        ([job(d_out=-1)], [V]),
        ([job(n=-3)], [V]),                               # negative batch
        ([job(n=1 << 31)], [V]),                          # batch beyond int range
        ([job(x=None)], [V]),                             # NULL input of a live job
        ([job(dy=None)], [G]),                            # gradient job without its dy rows
        ([job(lap=None)], [LAP]),                         # Laplacian job without its lap rows
        ([job(lap=None)], [ADV]),                         # advect job without its foot buffer
        ([job(lap=P[3])], [ADV]),                         # foot aliases f(x)
        ([job(d_out=1)], [ADV]),                          # advect needs f: R^d -> R^d
        ([job(), job(x=P[4], y=P[6], dy=P[7], lap=P[8])], [ADV, V]),  # the foot is another job's input
        ([job()], [ADV], None),                           # advect without its (dt, lo, hi)
        ([job()] * 7, [V] * 7),                           # more jobs than INSR_MAX_FWD_JOBS (6)
        ([job(n=0x40000000), job(n=0x40000000, x=P[5])], [V, V]),  # total beyond int range
    ]
    for case in bad:
        jobs, modes = case[0], case[1]
        args = {} if len(case) == 2 else {"scalars": case[2]}
        assert call(jobs, modes, **args) == -1, (modes, [(j.n, j.d_out) for j in jobs])
    assert call([job()], [V], prec=V | 1) == -1           # a jet mode inside prec_mode
    assert lib.insr_siren_jet_fwd_mixed(None, None, None, 1, 2, 2, 4, 128, 0, None) == -1


def test_value_backward_launch_shape(lib):
    """The x6 value backward at W = 128 runs about half as many blocks as CUs (each block's
    partial row is re-read by the reduction; capi.hip launch_shape, kbench r3d): 4,178 points
    -> 131 blocks of 2 tiles, 8,354 -> 131 of 4, 16,708 -> 209 balanced blocks of <= 5
    (256 CUs: the host answer without a GPU)."""
    V = 0
    assert (lib.insr_jet_split_tiles(4178, 2, 128, V, 1), lib.insr_jet_partial_blocks(4178, 2, 128, V)) == (2, 131)
    assert (lib.insr_jet_split_tiles(8354, 2, 128, V, 1), lib.insr_jet_partial_blocks(8354, 2, 128, V)) == (4, 131)
    assert (lib.insr_jet_split_tiles(16708, 2, 128, V, 1), lib.insr_jet_partial_blocks(16708, 2, 128, V)) == (5, 209)
    assert lib.insr_jet_partial_blocks(1000, 2, 128, V) == 63   # 63 tiles: one per block


def test_backward_path_policy(lib):
    """insr_jet_bwd_path answers on the host: the resident-dW path for the fluid nets' Laplacian
    backward from 4,096 points (its f16x3 saved-stream kernel while the INSR_BWD_F16_FUSED bit is on,
    else -- with bf16x6 products -- the two-kernel path below 32,768 points), two-kernel at W = 256, the fused kernel for value jets below 24,576 points
    (two-kernel from there), the resident-dW kernel for the fluid2DtlgnM value batch (from 49,152
    points) or when forced (policy 3); policy 4 forces the recompute backward (path 3: no saved
    streams) where it applies, independently of n (the forward's skip-the-saves decision must match
    the backward's); the per-call INSR_JET_POLICY bits force a path for A/B studies."""
    from base import _native as nat
    V, G, LAP = nat.MODE_VALUE, nat.MODE_GRAD, nat.MODE_LAP
    P = nat.jet_policy
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP) == 2
    assert lib.insr_jet_bwd_path(8192 + 163, 2, 1, 4, 128, LAP) == 2   # the fluid2DtlgnM 8-way shard
    assert lib.insr_jet_bwd_path(4096, 2, 1, 4, 128, LAP) == 2
    assert lib.insr_jet_bwd_path(4095, 2, 1, 4, 128, LAP) in (0, 1)
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP | nat.jet_bwd_f16(3)) == 1  # bf16x6 resident: >= 32,768
    assert lib.insr_jet_bwd_path(16708, 2, 2, 4, 128, V) == 0
    assert lib.insr_jet_bwd_path(1024, 2, 2, 4, 128, V) == 0
    # fluid2DtlgnM: the two-kernel f16x3 Laplacian backward (resident when its products are bf16x6)
    assert lib.insr_jet_bwd_path(65536 + 1308, 2, 1, 4, 128, LAP) == 2
    assert lib.insr_jet_bwd_path(65536 + 1308, 2, 1, 4, 128, LAP | nat.jet_bwd_f16(0)) == 2
    assert lib.insr_jet_bwd_path(65536 + 1308, 2, 2, 4, 128, V) == 2
    assert lib.insr_jet_bwd_path(33092, 2, 2, 4, 128, V) == 1   # value jets two-kernel from 24,576
    assert lib.insr_jet_bwd_path(24000, 2, 2, 4, 128, V) == 0
    assert lib.insr_jet_bwd_path(32768, 3, 3, 5, 256, G) == 1
    # 5 hidden layers: the 2-d gradient jet (el2D's Jacobian) takes the saved-stream resident sweep from 4,096
    # points (round 6); value / Laplacian jets of that depth and the recompute kernel are not served by it
    assert lib.insr_jet_bwd_path(20400, 2, 2, 5, 128, G) == 2
    assert lib.insr_jet_bwd_kernel(20400, 2, 2, 5, 128, G) == 1
    assert lib.insr_jet_bwd_path(4095, 2, 2, 5, 128, G) not in (2, 3)
    assert lib.insr_jet_bwd_path(20400, 2, 2, 5, 128, V) not in (2, 3)
    assert lib.insr_jet_bwd_path(20400, 2, 1, 5, 128, LAP) not in (2, 3)
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP | nat.jet_prec(nat.PREC_BF16)) not in (2, 3)
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP | P(2)) == 1
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP | P(1)) == 0
    assert lib.insr_jet_bwd_path(17, 2, 1, 4, 128, LAP | P(3)) == 2
    assert lib.insr_jet_bwd_path(17, 2, 1, 3, 128, LAP | P(3)) != 2         # 4 hidden layers only
    assert lib.insr_jet_bwd_path(17, 2, 1, 4, 64, LAP | P(3)) != 2          # W = 128 only
    for n in (1, 17, 16708, 65536 + 1308):
        assert lib.insr_jet_bwd_path(n, 2, 1, 4, 128, LAP | P(4)) == 3
    assert lib.insr_jet_bwd_path(17, 2, 2, 4, 128, V | P(4)) == 3
    assert lib.insr_jet_bwd_path(17, 2, 2, 4, 128, G | P(4)) == 3
    assert lib.insr_jet_bwd_path(16708, 1, 1, 4, 128, LAP | P(4)) != 3        # 1-d Laplacian: 3 streams
    assert lib.insr_jet_bwd_path(16708, 2, 1, 3, 128, LAP | P(4)) != 3        # 4 hidden layers only
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 64, LAP | P(4)) != 3         # W = 128 only
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP | P(4) | nat.jet_prec(nat.PREC_BF16)) != 3  # fp32-level only
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP) == 2              # no state left behind
    # malformed knob fields are refused like any bad mode
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP | (7 << nat.MODE_POLICY_SHIFT)) == -1
    assert lib.insr_jet_bwd_path(16708, 2, 1, 4, 128, LAP | (9 << nat.MODE_F16_SHIFT)) == -1


def test_multi_backward_plan(lib):
    """insr_siren_jet_bwd_grad_multi's plan, answered on the host: the value jobs of one
    network's loss.backward() -- the fluid interior (16,384 points) and its two 162-point wall
    bands -- share ONE fused launch whose blocks follow the balanced 5-tile shape of their combined
    batch (1024 tiles -> 205 blocks, 11 tiles -> 3 blocks each: 211 partial rows); a job whose own
    size takes another backward path keeps that path's workspace; malformed job lists are refused."""
    import ctypes
    from base import _native as nat
    V, LAP = nat.MODE_VALUE, nat.MODE_LAP
    stride = lib.insr_jet_partial_stride(2, 2, 4, 128)

    def work(ns, din=2, dout=2, mode=V):
        arr = (ctypes.c_long * len(ns))(*ns)
        return lib.insr_jet_bwd_multi_work_bytes(arr, len(ns), din, dout, 4, 128, mode)

    assert work([16384, 162, 162]) == 211 * stride * 4
    assert work([16384]) == lib.insr_jet_bwd_work_bytes(16384, 2, 2, 4, 128, V)
    assert work([162, 0, 162]) == 22 * stride * 4  # 1-tile blocks (324 points), 11 per band
    # Laplacian interior: the two-kernel path alone; bands beside it in the fused launch
    lw = lib.insr_jet_bwd_work_bytes(16708, 2, 1, 4, 128, LAP)
    pw = work([162, 162], dout=1, mode=LAP)
    assert work([16708, 162, 162], dout=1, mode=LAP) == max(lw, pw)
    for bad in ([], [-1], [1] * (nat.MAX_BWD_JOBS + 1), [1 << 31]):
        assert work(bad) == -1, bad
    assert lib.insr_siren_jet_bwd_grad_multi(None, 1, 2, 2, 4, 128, V, None, None, None, 0, None) == -1
    jobs = (nat.BwdJob * 1)(nat.BwdJob(None, None, None, None, None, 64))  # live job without x / act
    assert lib.insr_siren_jet_bwd_grad_multi(jobs, 1, 2, 2, 4, 128, V, 1, 1, 1, 0, None) == -1


def test_weight_plane_layout_matches_python(lib):
    """base.MLP sizes its flat storage [parameters | pad | planes | status quad] itself (no library call
    on the CPU path): both sizes must equal the library's (an undersized store would put the fp16 range
    guard's status word past the allocation)."""
    import base
    for din, dout, L, W in ((2, 1, 4, 128), (2, 2, 4, 128), (3, 3, 5, 256), (1, 1, 3, 64), (2, 2, 5, 68)):
        net = base.MLP(din, dout, L, W, nonlinearity="sine")
        kw = net.kernel_width
        assert net.wsplit_offset() == lib.insr_siren_wsplit_offset(din, dout, L, kw)
        assert net.wsplit_floats() == lib.insr_siren_wsplit_floats(L, kw)
        assert net._store.numel() == lib.insr_siren_wsplit_offset(din, dout, L, kw) + lib.insr_siren_wsplit_floats(L, kw)
