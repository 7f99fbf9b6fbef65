"""bench.py's N-GPU argument path (CPU): `--gpus N` without a launcher starts N rank processes (one per GPU) with the
environment torch.distributed.run exports, before the parent touches any GPU; a failing rank's exit code comes back;
the spg_multi leg's device list follows the ranks' devices."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_envs():
    envs = bench.rank_envs(3, 29999, base={"HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999" for e in envs)
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)


class _FakeProc:
    def __init__(self, rc):
        self.rc = rc
        self.killed = False

    def poll(self):
        return self.rc

    def terminate(self):
        self.killed = True

    def kill(self):
        self.killed = True

    def wait(self):
        return self.rc


def _run_main(monkeypatch, argv, rcs):
    calls = []

    def fake_popen(cmd, env=None, **kw):
        calls.append((cmd, env))
        return _FakeProc(rcs[len(calls) - 1])

    monkeypatch.setattr(bench.subprocess, "Popen", fake_popen)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    with pytest.raises(SystemExit) as ex:
        bench.main()
    return ex.value.code, calls


def test_gpus_without_launcher_spawns_ranks(monkeypatch):
    code, calls = _run_main(monkeypatch, ["--gpus", "2", "--backend", "gloo", "--legs", "none"], [0, 0])
    assert code == 0
    assert len(calls) == 2
    for r, (cmd, env) in enumerate(calls):
        assert cmd[0] == sys.executable and cmd[1].endswith("bench.py")
        assert cmd[2:] == ["--gpus", "2", "--backend", "gloo", "--legs", "none"]
        assert env["RANK"] == str(r) and env["LOCAL_RANK"] == str(r) and env["WORLD_SIZE"] == "2"
        assert env["MASTER_ADDR"] == "127.0.0.1"
    assert calls[0][1]["MASTER_PORT"] == calls[1][1]["MASTER_PORT"]


def test_failing_rank_exit_code(monkeypatch):
    code, calls = _run_main(monkeypatch, ["--gpus", "3"], [0, 7, 0])
    assert len(calls) == 3 and code == 7


def test_real_ranks_fail_loudly_without_gpu():
    """Two real rank processes on this GPU-less host: each fails at its first GPU call and the parent exits non-zero
    (it never hangs waiting for a rank, and never times one GPU while claiming two)."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--legs", "none"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert '"n_gpus"' not in r.stdout


def test_multi_devices(monkeypatch):
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert bench.multi_devices(2, "gloo") == [0, 0]
    assert bench.multi_devices(4, "nccl") == [0, 1, 2, 3]
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    assert bench.multi_devices(3, "gloo") == [0, 1, 0]


def test_multi_helper_protocol():
    """Rank 0's multi-device helper: it touches nothing until it reads "go"; rank 0 collects its JSON line, and kills it
    (by PID) past the time limit, reporting the leg as timed out instead of losing the per-rank line."""
    ok = subprocess.Popen([sys.executable, "-c", "import sys, json; sys.stdin.readline(); print(json.dumps({'value': 3}))"],
                          stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    assert bench.run_helper(ok, 60) == {"value": 3}
    hang = subprocess.Popen([sys.executable, "-c", "import sys, time; sys.stdin.readline(); time.sleep(600)"],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    out = bench.run_helper(hang, 2)
    assert "did not finish" in out["error"] and hang.poll() is not None
    # a helper whose rank 0 goes away without the signal exits on its own
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--multi-helper", "--gpus", "2"], input="",
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and p.stdout == ""


def _full_result():
    """The r05 default run's full nested result (20.5 KB when printed whole: the line the driver could not parse)."""
    import json
    with open(os.path.join(ROOT, "profiles", "r05zy_final_bench", "bench.json")) as f:
        return json.load(f)


def test_compact_line_under_limit_and_complete(tmp_path, capsys):
    import json
    res = _full_result()
    assert len(json.dumps(res)) > 16000
    bench.emit(res, str(tmp_path / "detail_n{n}.json"))
    out = capsys.readouterr().out
    lines = out.splitlines()
    assert len(lines) == 1 and len(lines[0].encode()) < bench.LINE_LIMIT < 8192
    line = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "higher_is_better", "scaling", "vs_baseline", "data"):
        assert k in line, k
    assert line["value"] == pytest.approx(res["value"], rel=1e-5)
    assert line["ms_per_step"] == pytest.approx(res["ms_per_step"], rel=1e-5)
    rf = line["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rf)
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-3)
    assert {"value", "unit", "cores", "kind", "sample"} <= set(line["cpu_baseline"])
    for leg in ("parity_mode", "sars1k", "sars100k", "chr1_30x", "config4", "multi_device"):
        assert {"value", "ms_per_step", "frac"} <= set(line["legs"][leg]), leg
    assert line["legs"]["end_to_end"]["uncapped"]["process_bam_pos_s"] > 0
    # the full result is in the detail file, byte for byte what the run produced
    detail = tmp_path / "detail_n1.json"
    assert json.loads(detail.read_text()) == res
    assert line["detail"].endswith("detail_n1.json")


def test_compact_line_bounded_with_long_fields():
    import json
    res = _full_result()
    res["multi_device"] = {"error": "x" * 50000}
    res["config"]["workload"] = "w" * 3000
    res["end_to_end"]["uncapped"]["path"] = "p" * 50000
    s = json.dumps(bench.compact_line(res))
    assert len(s) < 8192
    assert json.loads(s)["value"] == pytest.approx(res["value"], rel=1e-5)
