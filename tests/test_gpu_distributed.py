"""bench.py's N > 1 path on the product, rehearsed on one GPU.

The driver runs `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` with one
rank per GPU over RCCL; `python bench.py --gpus N` alone starts the same N ranks itself (a child
torch.distributed.run).  RCCL refuses two ranks on one device, so this test runs the same
command with HPT_BENCH_BACKEND=gloo (bench.py's rehearsal switch: the ranks share the visible
GPU and the film is reduced from a host copy) -- everything else is the bench's own N > 1 path:
the environment rendezvous, each rank rendering its Hilbert-cyclic shard of 32x32 blocks through
libhairpt, the barrier + max-over-ranks timing and the reduce of the RGBW films to rank 0.
Rank 0 must print exactly one JSON line, for 2 GPUs, whose reduced frame equals the one-rank
frame up to summation order (the film fingerprint is the fp64 sum of the RGBW film).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--config", "straight_kk", "--width", "160", "--height", "96", "--spp", "16", "--steps", "2",
        "--warmup", "1", "--cpu-baseline", "off"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lines(res):
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    return [json.loads(l) for l in res.stdout.splitlines() if l.startswith('{"metric"')]


@pytest.mark.gpu
def test_bench_two_ranks_reduce_the_one_rank_frame(tmp_path):
    env = dict(os.environ, HPT_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    one = _lines(subprocess.run([sys.executable, "bench.py", "--gpus", "1",
                                 "--workdir", str(tmp_path / "w1")] + ARGS,
                                cwd=ROOT, env=env, capture_output=True, text=True, timeout=240))
    two = _lines(subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                                 "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                                 "--workdir", str(tmp_path / "w2")] + ARGS,
                                cwd=ROOT, env=env, capture_output=True, text=True, timeout=240))
    # no launcher: bench.py --gpus 2 starts its two ranks itself
    self_launched = _lines(subprocess.run([sys.executable, "bench.py", "--gpus", "2",
                                           "--workdir", str(tmp_path / "w3")] + ARGS,
                                          cwd=ROOT, env=env, capture_output=True, text=True, timeout=240))
    assert len(one) == 1 and len(two) == 1 and len(self_launched) == 1  # rank 0 alone prints, once
    a, b = one[0], two[0]
    assert a["n_gpus"] == 1 and b["n_gpus"] == 2 and b["steps"] == 2 and b["value"] > 0
    assert b["config"]["workload"] == a["config"]["workload"]
    # what the process group saw, not what the launcher claimed
    for x in (b, self_launched[0]):
        assert x["n_gpus"] == 2 and x["config"]["world_size"] == 2 and x["config"]["dist_backend"] == "gloo"
        assert x["config"]["gpus_arg"] == 2
    assert a["config"]["world_size"] == 1 and a["config"]["dist_backend"] is None
    assert abs(self_launched[0]["stats"]["film_fingerprint"] - b["stats"]["film_fingerprint"]) <= 1e-6 * abs(
        b["stats"]["film_fingerprint"])
    fa, fb = a["stats"]["film_fingerprint"], b["stats"]["film_fingerprint"]
    assert fa > 0 and abs(fa - fb) <= 1e-6 * fa, (fa, fb)
    # rank 0's own counters (its shard's camera rays) cover part of the frame
    assert 0 < b["stats"]["camera_rays_packet"] < a["stats"]["camera_rays_packet"]
