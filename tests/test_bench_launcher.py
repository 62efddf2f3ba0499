"""bench.py's launcher contract (CPU): `--gpus N` without a launcher starts N ranks through
torch.distributed.run before anything in the parent touches the GPU, and a rank refuses to run
when WORLD_SIZE disagrees with --gpus."""
import importlib.util
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_launcher_command_starts_n_ranks():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "2"]
    cmd = b.launcher_command(b.parse_args(argv), argv)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1:] == [os.path.join(REPO, "bench.py"), *argv]


@pytest.mark.parametrize("gpus,world,ok", [(None, "1", True), (None, "4", True), (4, "4", True), (8, "4", False),
                                           (2, "1", False)])
def test_check_world(gpus, world, ok):
    b = _bench()
    args = b.parse_args([] if gpus is None else ["--gpus", str(gpus)])
    if ok:
        assert b.check_world(args, {"WORLD_SIZE": world}) == int(world)
    else:
        with pytest.raises(SystemExit) as e:
            b.check_world(args, {"WORLD_SIZE": world})
        assert e.value.code == 2


def test_main_spawns_before_touching_the_gpu(monkeypatch):
    import torch
    b = _bench()
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(b.subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 7)
    monkeypatch.setattr(b, "run", lambda args: pytest.fail("the parent must not render"))
    with pytest.raises(SystemExit) as e:
        b.main(["--gpus", "2", "--spp", "4"])
    assert e.value.code == 7                      # the launcher's exit status
    (cmd, env), = calls
    assert "--nproc-per-node=2" in cmd and cmd[-4:] == ["--gpus", "2", "--spp", "4"]
    assert env.get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"
    assert not torch.cuda.is_initialized()


def test_defaults_are_the_baseline_workload():
    b = _bench()
    a = b.parse_args([])
    # N > 1 headline: the C4 1920x1080 frame strong-scaled over the ranks (the metric's resolution,
    # BASELINE.json north_star "1920x1080 ... at 1, 2, 4 and 8 GPUs"); weak scaling is a side field
    assert (a.gpus, a.config, a.scaling, a.walk, a.path) == (None, "c4", "strong", "ordered", "megakernel")
    assert b.parse_args(["--config", "c5"]).config == "c5"
    assert a.dispatch == 0   # the per-pass DispatchRay timing is opt-in, never the default line
