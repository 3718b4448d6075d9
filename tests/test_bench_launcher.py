"""bench.py --gpus N: the parent starts torch.distributed.run as a child
process before anything imports torch or touches a GPU (never exec), and the
ranks check that the world is the one asked for."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import json, subprocess, sys
sys.path.insert(0, %r)
import bench
seen = []
class R:
    returncode = 7
def fake_run(cmd, env=None, **kw):
    seen.append({"cmd": cmd, "ipc": env.get("HSA_ENABLE_IPC_MODE_LEGACY")})
    return R()
subprocess.run = fake_run
sys.argv = ["bench.py"] + %r
rc = bench.main()
print(json.dumps({"rc": rc, "seen": seen, "torch": "torch" in sys.modules}))
"""


def run_probe(argv, env=None):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    r = subprocess.run([sys.executable, "-c", PROBE % (REPO, argv)], capture_output=True, text=True, env=e,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1]), r


def test_parent_spawns_torchrun_child_without_torch():
    out, _ = run_probe(["--gpus", "4", "--steps", "3", "--warmup", "1"])
    assert out["torch"] is False            # the parent never imported torch (so never touched the GPU)
    assert out["rc"] == 7                    # the child's exit code is forwarded
    (call,) = out["seen"]
    cmd = call["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "3", "--warmup", "1"]   # argv passed through
    assert call["ipc"] == "0"


def test_sharded_modes_only():
    out, r = run_probe(["--gpus", "2", "--mode", "decode"])
    assert out["rc"] == 2 and out["seen"] == [] and out["torch"] is False
    assert "runs on one GPU" in r.stderr
    for mode in ("biobank", "distfile"):
        out, _ = run_probe(["--gpus", "2", "--mode", mode])
        assert len(out["seen"]) == 1 and out["torch"] is False


def test_inside_a_rank_no_relaunch():
    # WORLD_SIZE set (we are a rank): main() goes on to the bench itself; here
    # the world check rejects the mismatch before any GPU call
    import bench

    class A:
        gpus = 2
    try:
        bench.check_world(A, None, 4, 0, True)
    except RuntimeError as e:
        assert "WORLD_SIZE=4 but --gpus 2" in str(e)
    else:
        raise AssertionError("mismatch accepted")
    bench.check_world(A, None, 2, 1, True)    # rehearsal: both ranks on cuda:0, no device count needed


def test_launcher_argv_shape():
    import bench
    cmd = bench.launcher_argv(8, ["--gpus", "8"], 29511)
    assert cmd[-3:] == [os.path.join(REPO, "bench.py"), "--gpus", "8"]
    assert "--master-port=29511" in cmd
