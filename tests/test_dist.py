"""Multi-rank path of bench.py on CPU: world_size 2 over gloo (127.0.0.1).

Each rank is an independent stream shard (no data-path collective); the only
cross-rank traffic is the barrier and the max/sum reductions that turn per-rank work and time
into the whole-job rate.  GPU ranks use exactly this code (bench.Dist), one process per GPU.
"""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json
sys.path.insert(0, {root!r})
import bench
D = bench.Dist()
r = D.rank
D.barrier()
rate, tmax = bench.throughput(D, units_local=100.0 * (r + 1), seconds_local=1.0 + r)
print(json.dumps(dict(rank=r, world=D.world, rate=rate, tmax=tmax, mx=D.max(float(r)), sm=D.sum(1.0))), flush=True)
D.close()
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2])
def test_gloo_throughput_aggregation(world):
    import json
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER.format(root=ROOT)], env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        assert p.returncode == 0, e
        outs.append(json.loads(o.strip().splitlines()[-1]))
    units = sum(100.0 * (r + 1) for r in range(world))
    tmax = 1.0 + (world - 1)
    for o in outs:
        assert o["world"] == world
        assert o["tmax"] == tmax                      # max over ranks
        assert o["rate"] == pytest.approx(units / tmax)
        assert o["mx"] == world - 1 and o["sm"] == world


def test_single_rank_needs_no_torch():
    """N=1 never initialises torch.distributed (and so never loads torch's HIP runtime)."""
    code = f"import sys; sys.path.insert(0, {ROOT!r}); import bench; D = bench.Dist(); " \
           "print(D.dist is None, 'torch' in sys.modules)"
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert out.stdout.split() == ["True", "False"], out.stdout + out.stderr


def _bench_env():
    return {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                             "MASTER_ADDR", "MASTER_PORT")}


def test_gpus_n_spawns_n_ranks_without_a_launcher():
    """`python bench.py --gpus 2` (no torchrun) starts two fresh worker processes with RANK /
    LOCAL_RANK / WORLD_SIZE set, which meet over gloo on 127.0.0.1."""
    import json
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--probe-ranks"], env=_bench_env(), cwd=ROOT,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1                                # rank 0 prints the one line
    probe = json.loads(lines[0])["probe"]
    assert [p[:3] for p in probe] == [[0, 0, 2], [1, 1, 2]]
    assert probe[0][3] != probe[1][3]                     # two distinct processes


def test_gpus_n_without_devices_fails_instead_of_sharing():
    """No silent device sharing: ranks whose GPU is not visible end the run with a non-zero exit
    and no JSON line (here: no GPU at all)."""
    env = dict(_bench_env(), HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"],
                         env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode != 0
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_device_summary_counts_distinct_devices():
    import bench
    two = bench.device_summary([(1, 1, "0000:15:00.0"), (0, 0, "0000:05:00.0")])
    assert two["n_gpus"] == 2 and two["ranks"] == 2
    assert [d["rank"] for d in two["devices"]] == [0, 1]
    shared = bench.device_summary([(0, 0, "0000:05:00.0"), (1, 0, "0000:05:00.0")])   # --rehearse on one GPU
    assert shared["n_gpus"] == 1 and shared["ranks"] == 2
