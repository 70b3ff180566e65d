"""CPU test of bench.py's own rank launcher: `python bench.py --gpus N` with no
WORLD_SIZE in the environment starts N rank processes itself.  In this GPU-less container every rank
must start, fail before touching a device (pmc_device_count -> PMC_ERR_NODEV), and the parent must
exit non-zero promptly instead of falling back to a one-GPU run or hanging at the rendezvous."""
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU box: the launcher would start a real multi-GPU run")
@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks_and_fails_fast(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "1",
                        "--warmup", "0"], env=env, capture_output=True, text=True, timeout=240)
    dt = time.time() - t0
    err = p.stderr
    assert p.returncode != 0, (p.stdout, err)
    assert f"launched {n} rank processes" in err, err
    for r in range(n):
        assert f"rank {r}/{n}: starting" in err, err          # every rank process started
    assert "pmc_device_count -> -5" in err, err                 # PMC_ERR_NODEV, before any GPU call
    assert "exited with 3" in err, err
    assert not p.stdout.strip(), p.stdout                       # no bench line from a one-GPU fallback
    assert dt < 200, dt


def test_bench_world_size_set_does_not_relaunch():
    """Under an external launcher (WORLD_SIZE set) bench.py is a rank itself: no second launch."""
    src = open(os.path.join(REPO, "bench.py")).read()
    assert 'if args.gpus > 1 and "WORLD_SIZE" not in os.environ:' in src
