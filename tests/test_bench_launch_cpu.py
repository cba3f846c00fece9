"""CPU checks of bench.py's multi-rank contract: `bench.py --gpus N` with no launcher
environment starts N ranks itself (torch.distributed.run as a child process, never an exec), relays rank 0's JSON
line, and a rank whose WORLD_SIZE disagrees with --gpus fails loudly before touching the GPU."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def test_mismatched_gpus_fails_loudly():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "3", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "--gpus 3" in r.stderr and "WORLD_SIZE=2" in r.stderr
    with pytest.raises(SystemExit):
        bench.check_world(4, {"WORLD_SIZE": "8"})
    assert bench.check_world(8, {"WORLD_SIZE": "8"}) == 8
    assert bench.check_world(2, {}) is None


def test_launch_command_is_torchrun_child_of_this_script():
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "5"], 29500)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8" and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29500"
    assert cmd[-5:] == [os.path.abspath(bench.__file__), "--gpus", "8", "--steps", "5"]


def test_self_launch_relays_rank0_json_and_status(monkeypatch, capsys):
    """The parent streams the ranks' other output to stderr and prints exactly rank 0's JSON line; the launcher's
    exit status is returned (a fake launcher stands in for the GPU ranks here)."""
    line = {"metric": "m", "value": 1.0, "n_gpus": 2}
    prog = "import json,sys; print('rank log'); print(json.dumps(%r)); sys.exit(0)" % (line,)
    monkeypatch.setattr(bench, "launch_cmd", lambda gpus, argv, port: [sys.executable, "-c", prog])

    class A:
        gpus = 2
    assert bench.self_launch(A(), []) == 0
    out, err = capsys.readouterr()
    assert json.loads(out.strip()) == line and "rank log" in err
    monkeypatch.setattr(bench, "launch_cmd", lambda gpus, argv, port: [sys.executable, "-c", "import sys; sys.exit(3)"])
    assert bench.self_launch(A(), []) == 3


def test_local_grad_sync_takes_the_dp_path_without_a_collective():
    import torch
    from xuanpolicy_amd.distributed import LocalGradSync
    from xuanpolicy_amd.flat import FlatState
    net = torch.nn.Linear(3, 2)
    fs = FlatState(net.parameters())
    h = LocalGradSync(fs)
    before = fs.flat.clone()
    h(fs.params)
    assert h.calls == 1 and h.collectives == 0 and not h.begin(fs.params[0].grad)
    assert torch.equal(fs.flat, before)
