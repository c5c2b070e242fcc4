"""bench.py's N-GPU launch (no GPU needed): `python bench.py --gpus N` without a
launcher starts N ranks itself, one process per GPU, with the environment
torchrun would give them; it refuses to run on fewer GPUs than asked, and a
launcher's WORLD_SIZE must agree with --gpus.  The ranks then run the same
per-GPU job at every N (weak scaling)."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, env=env, timeout=timeout)


def test_dry_run_plans_one_rank_per_gpu():
    for n in (2, 4, 8):
        p = _run(["--gpus", str(n), "--steps", "3", "--warmup", "1", "--dry-run"])
        assert p.returncode == 0, p.stderr
        plan = json.loads(p.stdout.strip().splitlines()[-1])
        assert plan["world_size"] == n
        ranks = plan["ranks"]
        assert [int(r["RANK"]) for r in ranks] == list(range(n))
        assert [int(r["LOCAL_RANK"]) for r in ranks] == list(range(n))
        assert {r["WORLD_SIZE"] for r in ranks} == {str(n)}
        assert {r["MASTER_ADDR"] for r in ranks} == {"127.0.0.1"}
        assert len({r["MASTER_PORT"] for r in ranks}) == 1
        assert {r["HSA_ENABLE_IPC_MODE_LEGACY"] for r in ranks} == {"0"}
        # every worker runs this script with the caller's arguments (the same job at every rank)
        assert plan["argv"][1] == BENCH and plan["argv"][2:] == ["--gpus", str(n), "--steps", "3", "--warmup", "1",
                                                                 "--dry-run"]


def test_too_few_gpus_fails_loudly():
    # this container has no GPU: any N > 1 is more than the visible devices
    p = _run(["--gpus", "2", "--steps", "1"])
    assert p.returncode == 2
    assert "GPU(s) visible" in p.stderr and p.stdout == ""


def test_launcher_world_size_must_match():
    p = _run(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr


def _fake_kfd(root, n_gpus, n_cpus=2):
    """A KFD topology tree: CPU nodes (simd_count 0) first, then GPU nodes."""
    for i in range(n_cpus + n_gpus):
        d = root / str(i)
        d.mkdir(parents=True)
        simd = 0 if i < n_cpus else 1024
        (d / "properties").write_text(f"cpu_cores_count {0 if simd else 64}\nsimd_count {simd}\n"
                                      f"location_id {i * 8}\ndomain 0\n")
    (root / "not_a_node").mkdir()


def test_gpu_count_from_sysfs(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    _fake_kfd(tmp_path, 8)
    for v in bench.VISIBILITY_VARS:
        monkeypatch.delenv(v, raising=False)
    assert len(bench.kfd_gpus(str(tmp_path))) == 8
    assert bench.count_gpus(str(tmp_path)) == 8
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,3")
    assert bench.count_gpus(str(tmp_path)) == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")
    assert bench.count_gpus(str(tmp_path)) == 1
    assert bench.count_gpus(str(tmp_path / "missing")) == 0


def test_launcher_counts_gpus_from_sysfs(tmp_path):
    # the launcher process counts the devices from the KFD topology (no HIP call in the parent)
    _fake_kfd(tmp_path, 4)
    env = {"FASTKMER_KFD_TOPOLOGY": str(tmp_path)}
    p = _run(["--gpus", "4", "--steps", "1", "--dry-run"], env)
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout.strip().splitlines()[-1])["visible_gpus"] == 4
    p = _run(["--gpus", "8", "--steps", "1"], env)
    assert p.returncode == 2 and "only 4 GPU(s) visible" in p.stderr
