"""bench.py's refusals: runs that cannot give a valid bench line
exit non-zero and print no value.  No GPU needed: every refusal happens before the first GPU
call (device counting does not initialise HIP)."""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(args, **env):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                       env=e, timeout=300, cwd=REPO)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_gpus_more_than_visible_devices_fails_loudly():
    """--gpus 2 where fewer than 2 GPUs are visible (none here, one on a 1-GPU box): exit code 2,
    a message naming both numbers, and no bench value -- never a line with n_gpus < 2."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("this machine has >= 2 GPUs: --gpus 2 would really launch two ranks")
    rc, line, err = run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert rc == 2, err
    assert line is not None and line.get("value") is None and "n_gpus" not in line
    assert "--gpus 2" in line["error"]


def test_launcher_world_size_must_match_gpus():
    """Under a launcher (WORLD_SIZE set) with a different --gpus: refused, no value."""
    rc, line, err = run_bench(["--gpus", "1", "--steps", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert rc == 2, err
    assert line.get("value") is None and "launcher started 2" in line["error"]


@pytest.mark.parametrize("env", [{"DP_ABLATE": "side"}, {"DP_GEMM_DEBUG": "8192"}])
def test_ablation_or_debug_switch_refused(env):
    """DP_ABLATE / DP_GEMM_DEBUG make the frame invalid or change its schedule: no value
    (exit 3) unless the run is an explicit --ab timing run."""
    rc, line, err = run_bench(["--steps", "1"], **env)
    assert rc == 3, err
    assert line.get("value") is None and "use --ab" in line["error"]


def _timed_worker(rank, world, port, q):
    """One rank of bench.timed_steps over gloo with a stub model: frame k -> rank k mod world, the
    depth map of global frame k is a (3, 5) map filled with k; rank 1 is slower per frame."""
    import time

    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    import bench
    from depth_pro import distributed as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        steps, warmup = 5, 2
        mine = D.shard_frames((steps + warmup) * world, rank, world)
        calls = []

        def infer_one(n):
            calls.append(mine[n])
            if rank == 1:
                time.sleep(0.05)
            return torch.full((3, 5), float(mine[n])), ("status", mine[n])

        seen = []
        run = bench.timed_steps(infer_one, steps, warmup, world, torch.device("cpu"), sync=lambda: None,
                                on_gathered=lambda n, bufs: seen.append([t.clone() for t in bufs]))
        q.put((rank, run["elapsed"], run["frames_total"], [s[1] for s in run["statuses"]], calls,
               [int(t[0, 0]) for t in D.order_results(seen, world)] if rank == 0 else None))
    finally:
        dist.destroy_process_group()


def test_timed_steps_world2_gloo():
    """bench.py's N-rank path over gloo with world 2 and a stub model: the
    timed window is the MAX over ranks (rank 1 sleeps 50 ms per frame, so both ranks report
    >= 5 x 50 ms), frames_total = steps x world, every infer call's status is kept, each rank runs
    its own frames (k -> rank k mod 2: warm-up then timed), and rank 0 receives every frame's
    depth map by the asynchronous double-buffered gather, in stream order."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_timed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = {m[0]: m[1:] for m in (q.get(timeout=5) for _ in range(2))}
    (el0, ft0, st0, calls0, order), (el1, ft1, st1, calls1, _) = res[0], res[1]
    assert el0 == el1 and el0 >= 5 * 0.05                 # max over ranks, rank 1's sleeps included
    assert ft0 == ft1 == 10
    assert calls0 == [0, 2, 4, 6, 8, 10, 12] and calls1 == [1, 3, 5, 7, 9, 11, 13]
    assert st0 == calls0 and st1 == calls1                # one status per infer call, in order
    assert order == list(range(14))                       # warm-up + timed frames, stream order at rank 0
