"""Host-side cost of one bench timestep (diagnostic): the prev-net snapshot and the phase loops'
graph replays, timed on the host with the device idle before each call, next to the device time of
the same timestep (HIP events).  A timestep whose host work exceeds its device work is host-bound.

    python tools/host_timing.py --config advect1D [--reps 50]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "insr-pde_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="advect1D")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--iters", type=int, default=4)
    a = ap.parse_args()
    sys.argv = [sys.argv[0], f"--config={a.config}"]
    args = bench.parse()
    world, rank, _ = bench.setup_dist(args)
    model, cfg, wl, _ = bench.build_model(args, world, rank)
    loops = bench.phase_loops(model, wl)
    i = 0
    for _ in range(3):
        bench.run_steps(loops, i, 1)
        i += 1
    bench.run_timestep(model, wl, loops, i, a.iters)
    i += a.iters
    torch.cuda.synchronize()
    res = {}

    def host(name, fn):
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        ts.sort()
        res[name] = 1e6 * ts[len(ts) // 2]

    for p in range(len(loops)):
        host(f"snapshot[{p}]", lambda p=p: bench.snapshot(model, wl, p))
    sd = {}
    for p, pl in enumerate(loops):
        def rep(pl=pl):
            nonlocal i
            pl.run_iters(i, a.iters)
            i += a.iters
        host(f"run_iters[{pl.tag}] x{a.iters}", rep)
    if wl["pde"] == "fluid":
        net = model.velocity_field
    elif wl["pde"] == "advection":
        net = model.field
    else:
        net = model.deformation_field
    host("state_dict()", lambda: net.state_dict())
    sd = net.state_dict()
    prev = {"fluid": "velocity_field_prev", "advection": "field_prev"}.get(wl["pde"], "deformation_field_prev")
    host("load_state_dict(sd)", lambda: getattr(model, prev).load_state_dict(sd))
    # device time of one timestep
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dev = []
    for _ in range(10):
        torch.cuda.synchronize()
        e0.record()
        bench.run_timestep(model, wl, loops, i, a.iters)
        e1.record()
        i += a.iters
        torch.cuda.synchronize()
        dev.append(1e3 * e0.elapsed_time(e1))
    dev.sort()
    res[f"device timestep ({a.iters} iters/phase, host-launched from idle)"] = dev[len(dev) // 2]
    # each phase loop's group replay started from an idle device vs queued behind a previous replay
    for pl in loops:
        idle, b2b = [], []
        for _ in range(10):
            torch.cuda.synchronize()
            e0.record()
            pl.run_iters(i, a.iters)
            e1.record()
            i += a.iters
            torch.cuda.synchronize()
            idle.append(1e3 * e0.elapsed_time(e1))
            pl.run_iters(i, a.iters)
            i += a.iters
            e0.record()
            pl.run_iters(i, a.iters)
            e1.record()
            i += a.iters
            torch.cuda.synchronize()
            b2b.append(1e3 * e0.elapsed_time(e1))
        idle.sort()
        b2b.sort()
        res[f"replay[{pl.tag}] x{a.iters} from idle"] = idle[5]
        res[f"replay[{pl.tag}] x{a.iters} queued"] = b2b[5]
    for k, v in res.items():
        print(f"{k:60s} {v:9.1f} us", flush=True)


if __name__ == "__main__":
    main()
