"""bench.py --gpus N starts its own ranks (torch.distributed.run as a child process) when no
launcher did: rehearsed on the CPU with gloo (no GPU work), the rank-0 JSON line reports the
world size the process group really had."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_spawns_ranks_gloo_rehearsal():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse",
                          "--steps", "5", "--warmup", "1", "--backend", "gloo"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["process_group"]["world_size"] == 2
    assert sorted(rec["rank_devices"]) == [0, 1]
    assert rec["scaling"] == "weak"  # fluid2Dtlgn default; strong for the 8-GPU configs


def test_scaling_defaults():
    sys.path.insert(0, ROOT)
    import bench
    assert set(bench.STRONG_CONFIGS) == {"elasticity3Dbunny", "fluid2DtlgnM"}
