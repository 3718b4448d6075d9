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


def test_strong_summary():
    """The `strong` object of a --gpus N > 1 encode line: GT bytes of all
    ranks over the max-rank time, rows per rank summing to the dataset."""
    import bench
    per = [[125_000, 1_252_000_000, 85_000_000]] * 8
    s = bench.strong_summary(per, 0.02, 20, 0.25, 1_000_000, "chr22-shaped")
    assert s["rows_per_rank"] == [125_000] * 8 and s["gt_bytes_total"] == 8 * 1_252_000_000
    assert abs(s["value"] - 8 * 1_252_000_000 * 20 / 0.02 / 1e9) < 0.01 and s["ms_per_step"] == 1.0
    assert s["scaling"] == "strong" and s["unit"] == "GB/s"
    try:
        bench.strong_summary(per[:7], 0.02, 20, 0.25, 1_000_000, "x")
    except RuntimeError:
        pass
    else:
        raise AssertionError("lost rows accepted")


def test_rehearsal_line_carries_weak_and_strong():
    """profiles/r06/bench_n8_rehearsal.json: the driver's `python bench.py
    --gpus 8` path rehearsed on one GPU (8 gloo ranks on cuda:0,
    VCFC_BENCH_REHEARSAL=1): one JSON line holding the weak value and the
    strong split of the N=1 dataset (8 x 125k rows)."""
    p = os.path.join(REPO, "profiles", "r06", "bench_n8_rehearsal.json")
    if not os.path.exists(p):
        import pytest
        pytest.skip("no rehearsal record yet")
    line = [x for x in open(p).read().splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 8 and d["scaling"] == "weak" and d["value"] > 0
    assert d["rccl_world"]["world"] == 8
    st = d["strong"]
    assert st["rows_total"] == 1_000_000 and st["rows_per_rank"] == [125_000] * 8 and st["value"] > 0
    assert st["gt_bytes_total"] == 2504 * 4 * 1_000_000
