"""Headline benchmark: collocation-points/sec/timestep (incl. grad/Lap residual + Adam).

Workload (BASELINE.json configs[1]): fluid2Dtlgn -- SIREN 4x128
velocity (2->2) + pressure (2->1) networks, 128^2 = 16384 uniform-random interior
collocation points per phase iteration, Taylor-Green weights/dt as the reference.
One "step" = one inner iteration of EACH of the three phases of a fluid timestep
(_advect_velocity, _solve_pressure, _projection): fresh samples, fused HIP jets,
residual, HIP reverse jets, RCCL gradient all-reduce (N>1), fused Adam + plateau.
Each phase iteration is replayed from a hipGraph captured during warm-up.  The K timed steps
run as 5 timesteps in step() order: K/5 iterations of _advect_velocity, then
of _solve_pressure, then of _projection, with the prev-net snapshots between them; the line
carries the per-timestep times and their median / min / max throughput.

    value = (points per phase-iteration, all ranks) x 3 phases x K / max_rank(time)

Other BASELINE.json workloads (--config): fluid2DtlgnM (256^2 points), advect1D (one
_advect phase, 4096 points), elasticity2Dstretch (one _solve_deformation phase, 20000
points), elasticity3Dbunny (SIREN 5x256, 64^3 points); a step is one iteration of every
phase of that model's timestep.

Also reported: a roofline object for the dominant kernel (HIP events on its launch
stream, eager re-run of the same step after the timed region) and a CPU baseline
(the oracle restatement of the reference's torch graph, timed on this host).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling auto|strong|weak] [--config NAME]
  N > 1: one rank per GPU over RCCL.  Under torch.distributed.run (WORLD_SIZE set) the ranks
  are the launcher's; otherwise bench.py starts `python -m torch.distributed.run
  --nproc-per-node N` itself as a child process (before any GPU call) and exits with its code.
  --scaling auto (default): strong for elasticity3Dbunny and fluid2DtlgnM (the global batch
  split over the ranks, BASELINE.md "≥6× strong scaling" configs), weak otherwise.
  --rehearse: the launcher + process-group plumbing alone on the CPU (gloo), no GPU work.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md chip table: dense fp32 matrix peak (spec)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16 (no sparsity)
# per precision: (bench dtype, bf16 products per fp32-equivalent product, NQ of the kernel names)
PRECISION = {"fp32": ("fp32", 6, 3), "bf16x3": ("bf16x3", 3, 2), "bf16": ("bf16", 1, 1),
             # BASELINE configs[4] "mixed fp32/bf16 MFMA": bf16x3 forwards, bf16 backwards (the
             # dominant launch is a backward: its products and kernel names are the bf16 ones)
             "mixed": ("bf16x3/bf16", 1, 1)}
HBM_PEAK_GBS = 8000.0


T0 = time.time()


def log(msg):
    print(f"[bench {time.time() - T0:7.2f}s] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="fluid2Dtlgn", choices=sorted(WORKLOADS),
                    help="BASELINE.json workload (default: configs[1], the headline)")
    ap.add_argument("--scaling", choices=["auto", "strong", "weak"], default="auto")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--precision", choices=sorted(PRECISION), default="fp32",
                    help="matrix-core precision of every jet: fp32 (fp32-accurate split-bf16, the parity "
                         "config), bf16x3 (3 bf16 products), bf16 (1 product) or mixed (bf16x3 forwards, bf16 "
                         "backwards: BASELINE configs[4] 'mixed fp32/bf16 MFMA', within 1e-2)")
    ap.add_argument("--api", choices=["fused", "plain"], default="fused",
                    help="'plain' runs pde/fluid_plain.py / pde/advection_plain.py / pde/elasticity_plain.py, phase "
                         "bodies written only against the reference's base API (separate band samplers, torch "
                         "residuals and energies, lowered by the loop: base/lower.py) -- the drop-in case")
    ap.add_argument("--plain-line", choices=["auto", "on", "off"], default="auto",
                    help="also time the unchanged reference phase bodies (--api plain) after the fused run and add "
                         "them to the line as `plain` (auto: on for the default fluid2Dtlgn line on one GPU)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="one process runs the per-rank shard of a K-rank strong-scaling run (global batch / K "
                         "points per phase iteration; elasticity: the draw at resolution / K^(1/3)); 1 GPU")
    ap.add_argument("--warm-ms", type=float, default=200.0,
                    help="untimed timesteps (graph replays as in the timed region) for this long before timing")
    ap.add_argument("--graph-unroll", type=int, default=4,
                    help="iterations per hipGraph replay inside a timestep's phase loop (PhaseLoop "
                         "insr_graph_unroll; 1 = one replay per iteration)")
    ap.add_argument("--bwd-policy", type=int, default=0, choices=[0, 1, 2, 3, 4, 5],
                    help="backward path (A/B studies): 0 auto, 1 fused tile-split, 2 two-kernel, 3 resident dW, "
                         "4 recompute, 5 resident f16x3")
    ap.add_argument("--bwd-f16", type=int, default=-1, choices=list(range(-1, 8)),
                    help="x6 backward products on the fp16 matrix cores, INSR_BWD_F16_* mask (A/B studies; "
                         "-1 = library default)")
    ap.add_argument("--lib", default=None, help="an alternative build of libinsr_hip.so (same-box A/B studies only)")
    ap.add_argument("--cpu-seconds", type=float, default=25.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) or gloo (functional rehearsal)")
    ap.add_argument("--dp-path", action="store_true",
                    help="one process runs the data-parallel iteration itself (gradient arena, a world-1 RCCL "
                         "all-reduce between the two graphs, unfused sums + Adam): a rank's DP step measured on "
                         "one GPU (with --shard-of K: the K-rank strong run's rank step)")
    ap.add_argument("--frozen-ahead", action="store_true",
                    help="fluid: evaluate the frozen networks once per replayed group of U iterations "
                         "(base.sampling.frozen_ahead; A/B -- default: inside each iteration's mixed forward launch)")
    ap.add_argument("--frozen-stream", action="store_true",
                    help="fluid, with --frozen-ahead: that evaluation on a side stream (A/B)")
    ap.add_argument("--frozen-pipe", action="store_true",
                    help="fluid: frozen-network work per iteration on a side stream, one iteration ahead (A/B)")
    ap.add_argument("--no-seed-in-bwd", action="store_true",
                    help="launch every loss group (A/B studies; default: the fluid / advection bodies' groups are "
                         "evaluated inside the reverse jets, base/losses.py lazy_losses)")
    ap.add_argument("--no-defer-jets", action="store_true",
                    help="api plain: launch each network / diff-op call at once (A/B; default: the lowered body's "
                         "jets are queued and launched together at the first read, base/lower.py deferred_jets)")
    ap.add_argument("--no-advect-fused", action="store_true",
                    help="advect1D: the generic launches per iteration (A/B; default: one insr_advect1d_iteration "
                         "launch + the sums / Adam launch, base/advect_iter.py)")
    ap.add_argument("--rehearse", action="store_true",
                    help="CPU rehearsal of the multi-rank launch (gloo, no GPU work; tests)")
    args = ap.parse_args()
    if args.scaling == "auto":
        args.scaling = "strong" if args.config in STRONG_CONFIGS else "weak"
    return args


STRONG_CONFIGS = ("elasticity3Dbunny", "fluid2DtlgnM")


def launch_ranks(args):
    """--gpus N > 1 without a launcher: run torch.distributed.run with N local ranks as a CHILD
    process (nothing here has touched the GPU) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log("launching " + " ".join(cmd[2:8]) + " ...")
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rehearse:
        dev = local
        if world > 1:
            dist.init_process_group("gloo")
    else:
        ndev = torch.cuda.device_count()
        dev = local % max(ndev, 1)  # >1 rank per GPU only for functional rehearsal (--backend gloo)
        os.environ["LOCAL_RANK"] = str(dev)
        torch.cuda.set_device(dev)
        if world > 1:
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            else:
                dist.init_process_group(args.backend)
        elif args.dp_path:  # a world-1 process group: the DP iteration's own code, collective included
            import socket
            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(port))
            dist.init_process_group(args.backend, rank=0, world_size=1,
                                    **({"device_id": torch.device("cuda", dev)} if args.backend == "nccl" else {}))
    if world > 1:
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
        devs = [None] * world
        dist.all_gather_object(devs, dev)
        if args.backend == "nccl" and not args.rehearse:
            assert len(set(devs)) == world, f"ranks share a GPU: {devs}"
        args.rank_devices = devs
    else:
        args.rank_devices = [dev]
    return world, rank, local


# BASELINE.json configs: model class, phases of one step, interior points
# per phase iteration (global, before any sharding).  configs[1] fluid2Dtlgn is the default
# (headline) workload; the others are measured with --config.
WORKLOADS = {
    "fluid2Dtlgn": dict(pde="fluid", phases=("_advect_velocity", "_solve_pressure", "_projection"), res=128,
                        model="SIREN 4x128 velocity(2->2) + pressure(2->1)"),
    "fluid2DtlgnM": dict(pde="fluid", phases=("_advect_velocity", "_solve_pressure", "_projection"), res=256,
                         model="SIREN 4x128 velocity(2->2) + pressure(2->1), taylorgreen_multi"),
    "advect1D": dict(pde="advection", phases=("_advect",), res=4096, model="SIREN 3x64 field(1->1)"),
    "elasticity2Dstretch": dict(pde="elasticity", phases=("_solve_deformation",), res=100,
                                model="SIREN 5x128 deformation(2->2), arap+constraint+constraint_right+volume"),
    "elasticity3Dbunny": dict(pde="elasticity", phases=("_solve_deformation",), res=64,
                              model="SIREN 5x256 deformation(3->3), arap+kinematics+collision+external+volume "
                                    "(the reference's bunny volume, tests/golden/bunny_mesh.npz)"),
}


def interior_points(cfg, wl):
    """Global interior collocation points of one phase iteration."""
    if wl["pde"] == "fluid":
        return cfg.sample_resolution ** 2
    if wl["pde"] == "advection":
        return cfg.sample_resolution
    d = cfg.dim
    return sum(cfg.sample_resolution ** d for _ in cfg.sample_pattern)


def build_model(args, world, rank):
    import base
    from pde.config import baseline_config
    base._native.load(args.lib, check_build=args.lib is None)
    # the run's knobs (per-call mode bits of every jet this thread launches; none: library defaults)
    base._native.set_default_knobs(policy=args.bwd_policy or None, bwd_f16=None if args.bwd_f16 < 0 else args.bwd_f16)
    wl = WORKLOADS[args.config]
    res = wl["res"]
    cfg = baseline_config(args.config, sample_resolution=res, insr_graph=not args.no_graph, insr_dp_always=args.dp_path,
                          insr_graph_unroll=max(1, args.graph_unroll), insr_seed_in_bwd=not args.no_seed_in_bwd,
                          insr_defer_jets=not args.no_defer_jets, insr_frozen_ahead="pipe" if args.frozen_pipe else bool(args.frozen_ahead),
                          insr_frozen_stream=args.frozen_stream, insr_advect_fused=not args.no_advect_fused,
                          insr_sync_every=10 ** 9, insr_progress=False, early_stop=False,
                          proj_dir="/tmp/insr_bench", max_n_iters=10 ** 9,
                          insr_precision=None if args.precision == "fp32" else args.precision)
    n_global = interior_points(cfg, wl)
    if args.shard_of > 1:  # one rank's shard of a shard_of-rank strong-scaling run, measured alone
        if world != 1:
            raise SystemExit("--shard-of is a single-process measurement")
        if wl["pde"] in ("fluid", "advection"):
            cfg.insr_points_per_rank = n_global // args.shard_of
            return finish_model(args, cfg, wl, world, rank, n_global // args.shard_of)
        # elasticity: rank 0's share of the global draw through the strong-scaling code itself
        # (ElasticityModel._shard / _rows: each part's N / K rows drawn, nothing world-sized)
        cfg.insr_shard = (0, args.shard_of)
        return finish_model(args, cfg, wl, world, rank, n_global // args.shard_of)
    if wl["pde"] in ("fluid", "advection"):
        # strong: the global batch is split over ranks; weak: every rank keeps the full batch
        cfg.insr_points_per_rank = n_global // world if args.scaling == "strong" else n_global
    else:
        # elasticity draws the global batch and keeps its rank's slice (strong); weak: no slicing
        cfg.insr_dp_weak = args.scaling == "weak"
    return finish_model(args, cfg, wl, world, rank, n_global // world if args.scaling == "strong" else n_global)


def finish_model(args, cfg, wl, world, rank, per_rank):
    torch.manual_seed(1234)  # identical weights on every rank
    if wl["pde"] == "fluid" and args.api == "plain":
        from pde.fluid_plain import Fluid2DPlainModel as M
    elif wl["pde"] == "fluid":
        from pde.fluid import Fluid2DModel as M
    elif wl["pde"] == "advection" and args.api == "plain":
        from pde.advection_plain import Advection1DPlainModel as M
    elif wl["pde"] == "advection":
        from pde.advection import Advection1DModel as M
    elif args.api == "plain":
        from pde.elasticity_plain import ElasticityPlainModel as M
    else:
        from pde.elasticity import ElasticityModel as M
    model = M(cfg)
    model.timestep = 1
    model.init_cond_func = None
    torch.cuda.manual_seed(1234 + 7919 * rank)  # independent collocation points per rank
    return model, cfg, wl, per_rank


def phase_loops(model, wl):
    from base._loop import PhaseLoop
    loops = []
    for name in wl["phases"]:
        pl = PhaseLoop(model, getattr(type(model), name)._insr_phase, name, (), {})
        pl.start()
        loops.append(pl)
    return loops


def run_steps(loops, i0, k):
    out = None
    for i in range(i0, i0 + k):
        for pl in loops:
            out = pl.step(i)
    return out


def snapshot(model, wl, phase_idx):
    """The prev-net snapshots step() takes before a phase loop:
    fluid/model.py:64,69 (before the advection and the projection), advection/model.py:65,
    elasticity/model.py:122-123 -- in-place copies into the flat buffers (graph-safe)."""
    if wl["pde"] == "fluid" and phase_idx in (0, 2):
        model.velocity_field_prev.load_state_dict(model.velocity_field.state_dict())
    elif wl["pde"] == "advection" and phase_idx == 0:
        model.field_prev.load_state_dict(model.field.state_dict())
    elif wl["pde"] == "elasticity" and phase_idx == 0:
        model.deformation_field_prev_prev.load_state_dict(model.deformation_field_prev.state_dict())
        model.deformation_field_prev.load_state_dict(model.deformation_field.state_dict())


def run_timestep(model, wl, loops, i0, k):
    """One timestep in step() order: k iterations of each phase loop in turn,
    with the prev-net snapshots between them.  (The per-phase optimiser reset of the reference's
    loop is an O(1) cost per phase loop of max_n_iters iterations; the phase loops here keep
    their optimiser and hipGraphs across bench timesteps.)"""
    for p, pl in enumerate(loops):
        snapshot(model, wl, p)
        pl.run_iters(i0, k)  # groups of insr_graph_unroll iterations per graph replay


def sync_all(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
        torch.cuda.synchronize()


def macs_per_point(din, dout, L, W):
    """P = d_in W + L W^2 + W d_out multiply-accumulates per point per stream."""
    return din * W + L * W * W + W * dout


def jet_precision_names(precision):
    """The matrix-core PRODUCTS the jets actually run (forward / backward).  'fp32' is the fp32-level
    contract: f16x3 forwards; backwards whose contract is bf16x6 run f16x3 products on every path the
    INSR_JET_BWD_F16 mask covers and on the recompute path (always f16x3), bf16x6 products on the
    resident-dW kernel and on paths the mask leaves out."""
    from base import _native as nat
    if precision != "fp32":
        return {"mixed": "bf16x3/bf16"}.get(precision, precision)
    mask = nat.bwd_f16_mask()
    bwd = "f16x3" if mask == 7 else (f"bf16x6+f16x3(mask {mask})" if mask else "bf16x6")
    bwd += " (the bf16x6 resident-dW kernel of value jets >= 49,152 points: bf16x6)" if mask else ""
    return f"f16x3/{bwd}"  # the library's default pair: f16x3 forward, bf16x6-contract backward


def roofline(loops, n_local, precision="fp32"):
    """Eager re-run of one step with HIP events around every jet launch (on its launch stream)."""
    from base import _jet
    for pl in loops:  # eager path, same kernels and shapes as the captured graphs
        pl.use_graph = False
    _jet.TIMING["events"].clear()
    _jet.TIMING["on"] = True
    # the backward's sums in its own timed call (not held back for the Adam launch): a backward's time is
    # its sweep + its sums, as the dominant kernel's label says, without the Adam work the run fuses in
    _jet.DEFER_REDUCE = False
    reps = 5
    try:
        for _ in range(reps):
            run_steps(loops, 10 ** 6, 1)
        torch.cuda.synchronize()
    finally:
        _jet.DEFER_REDUCE = True
        _jet.TIMING["on"] = False
    agg = {}
    for key, e0, e1 in _jet.TIMING["events"]:
        agg.setdefault(key, []).append(e0.elapsed_time(e1))
    _jet.TIMING["events"].clear()
    per_step = {k: sum(v) / reps for k, v in agg.items()}
    # dominant kernel = the longest launch over the interior batch (boundary bands are ~1% of points;
    # a merged launch carries the interior plus its boundary / fixed points: n >= n_local)
    # (fused multi-network forwards, kind "fwdK", are listed in the table but not candidates)
    # (kind "iter": the one-launch advection iteration, base/advect_iter.py)
    dom = max((k for k in per_step if k[2] >= n_local and k[0] in ("fwd", "bwd", "iter")),
              key=lambda k: sum(agg[k]) / len(agg[k]))
    kind, mode, n, W, (din, dout, L) = dom
    ms = sum(agg[dom]) / len(agg[dom])
    # algorithmic flops per launch: 2P per point per stream per GEMM pass
    P = macs_per_point(din, dout, L, W)
    streams = {"value": 1, "grad": 1 + din, "lap": 2 + din}[mode]
    # an advection iteration launch: two fields' forward jets (1 pass each) + the trainable one's reverse (2)
    passes = {"fwd": 1, "bwd": 2, "iter": 4}[kind]
    flops = n * streams * passes * 2 * P
    achieved = flops / (ms * 1e-3) / 1e12
    table = {}
    for k, v in sorted(per_step.items(), key=lambda t: -t[1]):
        name = f"{k[0]}:{k[1]}:n{k[2]}:{k[4][0]}-{k[3]}x{k[4][2]}-{k[4][1]}"
        table[name] = round(table.get(name, 0.0) + v, 4)
    nq = PRECISION[precision][2]
    # the loss groups ride in the reverse jets (in-kernel seeds): the saved-stream backward's seeded instantiation
    seeded = bool(loops and loops[0].m._lazy_losses_on())
    kname, grid, x6, np_run = kernel_identity(kind, mode, n, din, dout, L, W, nq, seeded)
    traffic, tsrc = pmc_traffic(kname, grid)
    # peak = the dense matrix ceiling of the products the launch actually runs: its split kernels run NP
    # v_mfma_f32_16x16x32_{bf16,f16} (16 cyc, the ~2.5 PF dense rate) per fp32-level 16x16x32 MAC block
    # (NP = 6 bf16x6 / 3 f16x3 or bf16x3 / 1 bf16), i.e. 2500 / NP TFLOP/s of fp32-equivalent work
    # (= 157.3 x 16 / NP: the fp32 MFMA runs at 1/16 of the bf16 rate); achieved counts the algorithmic
    # fp32-equivalent flops, so frac <= 1 on every path and config
    np_ = np_run if x6 else None
    ceil = round(FP32_MFMA_PEAK_TFLOPS * 16.0 / np_, 1) if np_ else FP32_MFMA_PEAK_TFLOPS
    out = {"bound": "mfma", "achieved": round(achieved, 2), "peak": ceil, "unit": "TFLOP/s",
           "frac": round(achieved / ceil, 4), "traffic": traffic,
           "peak_basis": (f"dense fp16/bf16 matrix rate / {np_} products per fp32-level MAC (the products this launch "
                          f"runs; MI355X_MICROARCH.md: 157.3 TF fp32 = 1/16 of ~2.5 PF bf16/fp16)") if np_ else
                         "dense fp32 matrix peak (exact-fp32 v_mfma_f32_16x16x4_f32)",
           "traffic_unit": "bytes/launch (HBM: corrected FETCH_SIZE + WRITE_SIZE)", "traffic_source": tsrc,
           "kernel": f"{kname}{'' if isinstance(grid, list) else f' grid={grid}'} (n={n}, {din}->{dout} {L}x{W}, {mode} jet {kind})", "avg_ms": round(ms, 4),
           "algorithmic_gflop_per_launch": round(flops / 1e9, 3), "per_step_ms_by_launch": table,
           "fp32_matrix_peak": FP32_MFMA_PEAK_TFLOPS,
           "frac_of_fp32_matrix_peak": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4)}
    if np_:
        out["products_per_mac"] = np_
    return out


def kernel_identity(kind, mode, n, din, dout, L, W, nq=3, seeded=False):
    """The rocprof name and grid (threads) of the jet kernel the library picks for this launch, and
    the split products per fp32-equivalent MAC it runs (6 bf16x6, 3 f16x3 / bf16x3, 1 bf16).
    nq = 3 (the fp32-level precision): the forward runs f16x3 (template NQ = 4), the backward's
    products per the INSR_JET_BWD_F16 mask (NQ = 4 where on)."""
    from base import _native as nat
    lib = nat.lib()
    prec = {3: nat.PREC_BF16X6, 2: nat.PREC_BF16X3, 1: nat.PREC_BF16}[nq]
    m = {"value": nat.MODE_VALUE, "grad": nat.MODE_GRAD, "lap": nat.MODE_LAP}[mode]
    m_b = m | nat.jet_prec(prec) | nat.scope_bits()  # + the run's knobs (policy, f16 mask)
    S = {"value": 1, "grad": 1 + din, "lap": 2 + din}[mode]
    NT = W // 16
    lap = "true" if mode == "lap" else "false"
    f16 = nat.bwd_f16_mask() if nq == 3 else 0
    nprod = {4: 3, 3: 6, 2: 3, 1: 1}
    if kind == "iter":  # insr_advect1d_iteration: exact-fp32 products (v_mfma_f32_16x16x4_f32)
        nb = lib.insr_advect1d_rows(n)
        return f"insr::advect1d_iter_kernel<{L}>", nb * 512, False, 1  # (512 threads per block)
    path = lib.insr_jet_bwd_path(n, din, dout, L, W, m_b) if kind == "bwd" else 0
    if path == 3:  # the recompute backward (forward + reverse jet per tile, f16x3) + the fixed-order sums
        import ctypes
        thr = (ctypes.c_long * 3)()
        nat.check(lib.insr_jet_wide_launch_threads(n, din, dout, L, W, m_b, thr), "insr_jet_wide_launch_threads")
        zr = 4 if S == 1 else 2  # jet_fb.hip: hidden layers whose z-streams stay in registers
        parts = [(f"insr::jet_fb_x6<{S}, {lap}, {L}, {zr}, false>", thr[0]), ("insr::reduce_dw_kernel", thr[1])]
        return " + ".join(f"{k}|grid={g}" for k, g in parts) + " (recompute backward: forward + reverse jet per " \
            "tile in one persistent launch, no saved streams, then the dW / compact-row sums; time = both " \
            "launches; achieved counts the backward's algorithmic flops only, not the recomputed forward)", \
            parts, True, 3
    if path == 2 and lib.insr_jet_bwd_kernel(n, din, dout, L, W, m_b) == 1:
        # the resident-dW backward on jet_fb_x6's saved-stream variant (f16x3 products) + the sums
        import ctypes
        thr = (ctypes.c_long * 3)()
        nat.check(lib.insr_jet_wide_launch_threads(n, din, dout, L, W, m_b, thr), "insr_jet_wide_launch_threads")
        parts = [(f"insr::jet_fb_x6<{S}, {lap}, {L}, 1, true{', true' if seeded else ''}>", thr[0]),
                 ("insr::reduce_dw_kernel", thr[1])]
        return " + ".join(f"{k}|grid={g}" for k, g in parts) + " (resident-dW backward, f16x3: the reverse " \
            "sweep on the saved streams, dW in registers per CU, no adjoint round trip; then the dW / " \
            "compact-row sums; time = both launches)", parts, True, 3
    if path == 2:  # the resident-dW persistent kernel + the fixed-order sums
        import ctypes
        thr = (ctypes.c_long * 3)()
        nat.check(lib.insr_jet_wide_launch_threads(n, din, dout, L, W, m_b, thr), "insr_jet_wide_launch_threads")
        parts = [(f"insr::jet_bwd_x6r<{nq}, {S}, {lap}, {L}, 1>", thr[0]), ("insr::reduce_dw_kernel", thr[1])]
        return " + ".join(f"{k}|grid={g}" for k, g in parts) + " (resident-dW backward: persistent tile loop, " \
            "then the dW / compact-row sums; time = both launches)", parts, True, nprod[nq]
    if path == 1:  # two kernels + the dW sums
        import ctypes
        thr = (ctypes.c_long * 3)()
        nat.check(lib.insr_jet_wide_launch_threads(n, din, dout, L, W, m_b, thr), "insr_jet_wide_launch_threads")
        qp, qd = (4 if f16 & 2 else nq), (4 if f16 & 1 else nq)
        parts = [(f"insr::jet_bwd_x6p<{qp}, {NT}, {S}, {lap}>", thr[0]), (f"insr::dw_x6<{qd}, {NT}, {S}, {lap}>", thr[1]),
                 ("insr::reduce_dw_kernel", thr[2])]
        return " + ".join(f"{k}|grid={g}" for k, g in parts) + " (two-kernel backward: propagation, dW GEMM + row partials, sums; time = all three launches)", \
            parts, True, max(nprod[qp], nprod[qd])
    if kind == "bwd":
        T = lib.insr_jet_split_tiles(n, din, W, m_b, 1)
        nb = lib.insr_jet_partial_blocks(n, din, W, m_b)
        q = 4 if f16 & 4 else nq
    else:
        mf = (m | nat.scope_bits()) if nq == 3 else m_b  # the default forward precision (f16x3) serves the fp32-level runs
        T = lib.insr_jet_split_tiles(n, din, W, mf, 0)
        nb = ((n + 15) // 16 + T - 1) // T
        q = 4 if nq == 3 else nq
    return f"insr::jet_{kind}_x6<{q}, {NT}, {S}, {lap}, {T}>", nb * 64 * min(NT, 8), True, nprod[q]


def pmc_traffic(kname, grid):
    """HBM bytes per launch of this kernel from the committed rocprofv3 --pmc summary
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py from separate
    FETCH_SIZE / WRITE_SIZE passes of this benchmark); None if not profiled."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        tab = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    parts = grid if isinstance(grid, list) else [(kname, grid)]  # a multi-launch path: the sum of its launches
    tot = 0
    for name, g in parts:
        e = tab.get(f"{name}|grid={g}")
        if not e or "fetch_bytes" not in e or "write_bytes" not in e:
            return None, None
        tot += e["fetch_bytes"] + e["write_bytes"]
    return tot, tab.get("_source")


def cpu_baseline(config, seconds, n_rounds=3, iters=10):
    """The oracle (torch-CPU restatement of the reference graph) on this host's cores, over a
    bounded sample of the same workload (same nets, same phases; elasticity3Dbunny on a
    16384-point slice of its 262144-point batch: the per-point cost is size-independent)."""
    from oracle import siren_oracle as O
    from pde.config import baseline_config
    cores, share = cpu_threads()
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    wl = WORKLOADS[config]
    cfg = baseline_config(config, sample_resolution=wl["res"])
    L, W = cfg.num_hidden_layers, cfg.hidden_features

    def adam(nets):
        return O.OracleAdam([p for n in nets for p in n.parameters() if p.requires_grad], lr=1e-4)

    if wl["pde"] == "fluid":
        vel, vel_prev, pres = O.OracleSiren(2, 2, L, W), O.OracleSiren(2, 2, L, W), O.OracleSiren(2, 1, L, W)
        for p in vel_prev.parameters():
            p.requires_grad_(False)
        opts = [adam([vel, pres]) for _ in range(3)]
        N = cfg.sample_resolution ** 2
        nb = N // 100

        def X():
            return (torch.rand(N, 2) * 2 - 1).requires_grad_(True)

        def B(side):
            return O.sample_boundary2d_side(nb, side).requires_grad_(True)

        def one_step():
            O.update_step([vel, pres], O.fluid_advect_loss(vel, vel_prev, X(), B("horizontal"), B("vertical"),
                                                           cfg.dt), opts[0])
            O.update_step([vel, pres], O.fluid_pressure_loss(vel, pres, X(), B("horizontal"), B("vertical")),
                          opts[1])
            O.update_step([vel, pres], O.fluid_projection_loss(vel, vel_prev, pres, X(), B("horizontal"),
                                                               B("vertical")), opts[2])
        pts, what = 3 * N, f"3 phases x {N} pts"
    elif wl["pde"] == "advection":
        f, f_prev = O.OracleSiren(1, 1, L, W), O.OracleSiren(1, 1, L, W)
        for p in f_prev.parameters():
            p.requires_grad_(False)
        opt = adam([f])
        N = cfg.sample_resolution
        half = cfg.length / 2

        def one_step():
            x = ((torch.rand(N, 1) * 2 - 1) * half).requires_grad_(True)
            bc = O.sample_boundary1d(max(N // 100, 10)) * half
            O.update_step([f], O.advect1d_loss(f, f_prev, x, bc, cfg.dt, cfg.vel), opt)
        pts, what = N, f"1 phase x {N} pts"
    else:
        d = cfg.dim
        f, fp, fpp = O.OracleSiren(d, d, L, W), O.OracleSiren(d, d, L, W), O.OracleSiren(d, d, L, W)
        for n in (fp, fpp):
            for p in n.parameters():
                p.requires_grad_(False)
        opt = adam([f])
        vec = lambda *v: list(v[:d])  # noqa: E731
        ecfg = dict(dt=cfg.dt, energy=list(cfg.energy), ratio_arap=cfg.ratio_arap, ratio_volume=cfg.ratio_volume,
                    ratio_kinematics=cfg.ratio_kinematics, ratio_constraint=cfg.ratio_constraint,
                    ratio_collide=cfg.ratio_collide, plane_height=cfg.plane_height,
                    external_force=vec(cfg.external_force_x, cfg.external_force_y, cfg.external_force_z),
                    constraint_offset_right=vec(cfg.constraint_right_offset_x, cfg.constraint_right_offset_y,
                                                cfg.constraint_right_offset_z),
                    circle_center=vec(cfg.collide_circle_x, cfg.collide_circle_y, cfg.collide_circle_z),
                    circle_radius=cfg.collide_circle_radius, external_force_timesteps=cfg.external_force_timesteps)
        full = interior_points(cfg, wl)
        N = full if full <= 32768 else 16384  # el3D: a slice (per-point cost is independent of N)
        R = cfg.sample_resolution

        def one_step():
            parts = []
            for sp in cfg.sample_pattern:
                parts.append(torch.rand(R ** d, d) * 2 - 1 if sp == "random" else O.sample_uniform(R, d))
            x = torch.cat(parts)[:N].clone().requires_grad_(True)
            fixed = [torch.cat([torch.full((R, 1), s), torch.rand(R, d - 1) * 2 - 1], 1) for s in (-1.0, 1.0)]
            O.update_step([f], O.elasticity_loss(f, fp, fpp, x, fixed[0], fixed[1], ecfg), opt)
        pts = N
        what = f"1 phase x {N} pts" + (f" (slice of the {full}-point batch; points/s scaled as per-point "
                                        f"cost independent of the batch size)" if N < full else "")

    for _ in range(2):  # 2 warm-up iterations, then the median of 10 or more
        one_step()
    # the box's CPU share is a CFS quota on a shared host (tools/cpu_leg_study.py, profiles/r06/r6b/
    # cpustudy.jsonl): iteration times spread 1.5-2.3x whatever the thread count or pinning, so the sample is
    # as many iterations as the budget allows (>= 10) and the line carries the median, the fastest iteration
    # and both spreads (max / min, and p90 / p10 of the middle 80 %)
    times = []
    t_all = time.perf_counter()
    while len(times) < max(10, n_rounds * iters) and (len(times) < 10 or time.perf_counter() - t_all < seconds):
        t0 = time.perf_counter()
        one_step()
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_all > seconds and len(times) >= 3:  # bounded sample
            break
    times.sort()
    dt = times[len(times) // 2]
    p10, p90 = times[len(times) // 10], times[min(len(times) - 1, (9 * len(times)) // 10)]
    return {"value": round(pts / dt, 1), "value_min_time": round(pts / times[0], 1),
            "unit": "collocation-points/s", "cores": cores, "kind": "port", "cpu_share": share,
            "cpu_model": cpu_model(), "statistic": f"median of {len(times)} iterations after 2 warm-up",
            "spread_max_over_min": round(times[-1] / times[0], 3), "spread_p90_over_p10": round(p90 / p10, 3),
            # the explicit uncertainty of `value`: the sample's iteration rates span median x (1 +- u)
            "uncertainty_pct": round(50.0 * (times[-1] - times[0]) / dt, 1),
            "sample": f"oracle/siren_oracle.py {config}: {what}, torch CPU autograd + Adam, "
                      f"{torch.get_num_threads()} threads, median {dt * 1e3:.1f} ms/iter "
                      f"(min {times[0] * 1e3:.1f}, p10 {p10 * 1e3:.1f}, p90 {p90 * 1e3:.1f}, max {times[-1] * 1e3:.1f})"}


def cpu_threads():
    """(threads, share description) of the CPU leg.  The box exports OMP_NUM_THREADS = its CPU share and
    limits the container by a CFS quota (cgroup cpu.max, 16 CPUs of a 256-CPU host) while the affinity lists
    every CPU: with as many busy threads as the quota the process is throttled (16 threads: fastest
    iteration 425-436 ms; 12 threads: 308 ms, profiles/r06/r6b/cpustudy.jsonl), so the leg uses 3/4 of the
    quota."""
    omp = int(os.environ.get("OMP_NUM_THREADS", "1024"))
    cores = min(len(os.sched_getaffinity(0)), omp)
    share = f"affinity {len(os.sched_getaffinity(0))} CPUs, OMP_NUM_THREADS {os.environ.get('OMP_NUM_THREADS')}"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = int(quota) / int(period)
            share += f", cgroup quota {q:g} CPUs"
            cores = max(1, min(cores, int(q * 3 // 4)))
    except (OSError, ValueError):
        pass
    return cores, share


def cpu_model():
    """`lscpu` model name of this host."""
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:  # pragma: no cover - depends on the host
        pass
    return None


def rehearse(args, world, rank):
    """The multi-rank plumbing on the CPU: barrier-bracketed timed region, max over ranks,
    one JSON line from rank 0 (no GPU work; value = timed barriers per second)."""
    for _ in range(args.warmup):
        if world > 1:
            dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if world > 1:
            dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "rehearsal (no GPU work)", "value": round(args.steps / max(float(el), 1e-9), 1),
                          "unit": "barriers/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "scaling": args.scaling, "rank_devices": args.rank_devices,
                          "process_group": {"backend": "gloo", "world_size": world},
                          "config": {"workload": args.config}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def measure(args, model, wl, world):
    """Warm-up (eager iteration, graph captures, one timestep in step() order, the U-iteration group
    graphs, --warm-ms of sustained replays), then the timed region: --steps iterations of every phase as
    up to 5 timesteps.  Returns (phase loops, elapsed s (max over ranks), per-timestep ms, iterations per
    timestep, effective warm-up iterations)."""
    loops = phase_loops(model, wl)
    # iteration 0 runs eagerly, iteration 1 captures the hipGraphs: both must be warm-up,
    # so at least 2 untimed iterations run even when --warmup < 2 (reported as warmup_effective)
    w_eff = max(args.warmup, 0 if args.no_graph else 2, 1)
    for i in range(w_eff):
        run_steps(loops, i, 1)
        torch.cuda.synchronize()
        log(f"warmup step {i} done" + "".join(f" [{pl.tag}: capture failed {pl.capture_error}]"
                                              for pl in loops if getattr(pl, "capture_error", None)))
    # one more untimed step as a timestep in step() order (the prev-net snapshots, then each phase
    # loop in turn), so the timed region's first timestep is not the first use of that sequence
    run_timestep(model, wl, loops, w_eff, 1)
    torch.cuda.synchronize()
    w_eff += 1
    # and, with --graph-unroll U > 1, one untimed timestep of U iterations per phase: it captures
    # (and so runs) each phase loop's U-iteration graph outside the timed region
    U = max(1, args.graph_unroll)
    if U > 1 and not args.no_graph:
        run_timestep(model, wl, loops, w_eff, U)
        torch.cuda.synchronize()
        w_eff += U
    # sustained untimed timesteps (the graphs replayed as in the timed region) until --warm-ms of wall
    # time has passed: the timed region then starts with the replays warm and the device clocks at their
    # sustained level (without it the first timed timesteps run slower, profiles/r05/warm/)
    k_warm = U if (U > 1 and not args.no_graph) else 1
    t_warm = time.perf_counter()
    while (time.perf_counter() - t_warm) * 1e3 < args.warm_ms:
        run_timestep(model, wl, loops, w_eff, k_warm)
        w_eff += k_warm
        torch.cuda.synchronize()
    # timed region: --steps iterations of every phase, as `nts` timesteps in step() order
    # (K iterations per phase, phases in order, median of 5 timesteps); no loss
    # reads inside (sync_every = 1e9) and no host sync at the timestep boundaries either: the
    # per-timestep times come from HIP events recorded there, and the host's snapshot work
    # overlaps the device's previous timestep as it does in a run
    nts = max(1, min(5, args.steps))
    ks = [args.steps // nts + (1 if t < args.steps % nts else 0) for t in range(nts)]
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(nts + 1)]
    sync_all(world)
    t0 = time.perf_counter()
    evs[0].record()
    i = w_eff
    for t, k in enumerate(ks):
        run_timestep(model, wl, loops, i, k)
        evs[t + 1].record()
        i += k
    sync_all(world)
    elapsed = time.perf_counter() - t0
    ts_ms = [evs[t].elapsed_time(evs[t + 1]) for t in range(nts)]
    t = torch.tensor([elapsed] + ts_ms, device="cuda", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, ts_ms = float(t[0]), [float(v) for v in t[1:]]
    log(f"timed {args.steps} steps ({nts} timesteps): {elapsed * 1e3:.2f} ms")
    for pl in loops:  # which replay form each phase loop ended up with
        log(f"  {pl.tag}: graph {pl.graph is not None}, unroll {pl.unroll}, group graph {pl.graphU is not None}"
            + (f", capture error {pl.capture_error}" if getattr(pl, "capture_error", None) else ""))
    return loops, elapsed, ts_ms, ks, w_eff


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world, rank, local = setup_dist(args)
    log(f"world={world} rank={rank}")
    if args.rehearse:
        return rehearse(args, world, rank)
    model, cfg, wl, n_local = build_model(args, world, rank)
    from base import _native
    bwd_f16 = _native.bwd_f16_mask()  # the backward products on fp16 matrix cores in effect
    nph = len(wl["phases"])
    log(f"model built, {n_local} points per rank per phase")
    loops, elapsed, ts_ms, ks, w_eff = measure(args, model, wl, world)
    nts = len(ks)
    # points all ranks processed: strong = the global batch, weak = world x the per-rank batch
    n_all = interior_points(cfg, wl) if (args.scaling == "strong" and args.shard_of == 1) else n_local * world
    total_points = n_all * nph * args.steps
    value = total_points / elapsed
    per_ts = sorted((n_all * nph * k) / (ms * 1e-3) for k, ms in zip(ks, ts_ms))
    result = {
        "metric": "collocation-points/sec/timestep (incl. ∇/Δ residual + Adam) at 1/2/4/8 GPUs",
        "value": round(value, 1), "unit": "collocation-points/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "warmup_effective": w_eff, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None, "dtype": PRECISION[args.precision][0],
        "data": "synthetic (uniform-random "
        "collocation points, seeded SIREN init; no dataset exists for this path)",
        "config": {"workload": args.config, "model": wl["model"],
                   "points_per_phase_iter": n_all, "phases": nph, "global_batch": n_all,
                   "seq_len": None, "parallelism": f"dp{world}", "graph": not args.no_graph,
                   "precision": args.precision, "api": args.api, "sync_every": cfg.insr_sync_every,
                   "graph_unroll": 1 if args.no_graph else max(1, args.graph_unroll), "warm_ms": args.warm_ms,
                   "jet_precision": jet_precision_names(args.precision),
                   "bwd_policy": args.bwd_policy, "shard_of": args.shard_of, "dp_path": args.dp_path,
                   "seeds_in_bwd": bool(getattr(cfg, "insr_seed_in_bwd", True)),
                   "advect_fused": bool(getattr(model, "_fused_iteration_ok", lambda: False)()),
                   "frozen_ahead": bool(getattr(cfg, "insr_frozen_ahead", False)) and wl["pde"] == "fluid"
                   and args.api == "fused", "frozen_stream": bool(args.frozen_stream), "frozen_pipe": bool(args.frozen_pipe),
                   "lowered": bool(model._lower_on()), "deferred_jets": bool(model._defer_on()),
                   "bwd_f16": bwd_f16,
                   "timestep_order": f"{nts} timesteps x ({'/'.join(str(k) for k in ks)}) iterations per phase, "
                                     "phases in step() order with the prev-net snapshots; per-timestep times from HIP events"},
        "timesteps": {"count": nts, "iters_per_phase": ks, "ms": [round(v, 3) for v in ts_ms],
                      "value_median": round(per_ts[len(per_ts) // 2], 1), "value_min": round(per_ts[0], 1),
                      "value_max": round(per_ts[-1], 1)},
        "process_group": {"backend": args.backend if (world > 1 or args.dp_path) else None, "world_size": world,
                          "rank_devices": args.rank_devices},
    }
    if not args.no_roofline:  # every rank runs the eager steps (they contain the all-reduce)
        roof = roofline(loops, n_local, args.precision)
        if rank == 0:
            result["roofline"] = roof
        log("roofline done")
    plain_on = args.plain_line == "on" or (args.plain_line == "auto" and args.config == "fluid2Dtlgn")
    if plain_on and world == 1 and args.api == "fused" and args.shard_of == 1:
        # the drop-in number, driver-timed: the reference's phase bodies as written (pde/*_plain.py) on the
        # same kernels, through the loop's lowering and deferred jets, same steps / warm-up / timing
        pargs = argparse.Namespace(**vars(args))
        pargs.api = "plain"
        pmodel, _, _, _ = build_model(pargs, world, rank)
        log("plain model built")
        _, p_el, p_ts, p_ks, _ = measure(pargs, pmodel, wl, world)
        p_val = n_all * nph * args.steps / p_el
        p_per_ts = sorted((n_all * nph * k) / (ms * 1e-3) for k, ms in zip(p_ks, p_ts))
        result["plain"] = {"value": round(p_val, 1), "ms_per_step": round(p_el / args.steps * 1e3, 4),
                           "value_median_timestep": round(p_per_ts[len(p_per_ts) // 2], 1),
                           "vs_fused": round(p_val / value, 3), "lowered": bool(pmodel._lower_on()),
                           "model": f"pde/{wl['pde']}_plain.py: the reference's phase bodies as written "
                                    "(reference base API only; base/lower.py lowers them)"}
        log(f"plain line {p_val / 1e6:.1f} M pts/s")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        log("cpu baseline done")
        result["speedup_vs_cpu_baseline"] = round(value / result["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
