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


@pytest.mark.parametrize("env", [{"DP_ABLATE": "side"}, {"DP_GEMM_DEBUG": "8192"}, {"DP_SIDE_GATE": "fc2:fc1"},
                                 {"DP_LN_FOLD": "0"}])
def test_ablation_or_debug_switch_refused(env):
    """DP_ABLATE / DP_GEMM_DEBUG make the frame invalid or change its schedule: no value
    (exit 3) unless the run is an explicit --ab timing run."""
    rc, line, err = run_bench(["--steps", "1"], **env)
    assert rc == 3, err
    assert line.get("value") is None and "use --ab" in line["error"]
