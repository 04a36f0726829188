"""bench.py's own launcher: `python bench.py --gpus N` with no torchrun around it starts N
rank processes (before any GPU call) instead of timing one GPU; a launcher whose WORLD_SIZE
disagrees with --gpus ends the run; the first failing rank ends the job. CPU only (gloo)."""
import subprocess
import sys
import textwrap
import time

import pytest

from conftest import ROOT

sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_launch_decision():
    assert bench.launch_decision(1, {}) == "run"
    assert bench.launch_decision(8, {}) == "spawn"
    assert bench.launch_decision(2, {"WORLD_SIZE": "2", "RANK": "1"}) == "run"
    assert bench.launch_decision(1, {"WORLD_SIZE": "1"}) == "run"  # CUBIT_BENCH_DIST1 rehearsal under torchrun
    assert bench.launch_decision(8, {"WORLD_SIZE": "1"}).startswith("error")
    assert bench.launch_decision(1, {"WORLD_SIZE": "4"}).startswith("error")
    assert bench.launch_decision(0, {}).startswith("error")


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return p


def test_spawn_ranks_form_one_gloo_group(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    s = _script(tmp_path, f"""
        import os, sys
        import torch, torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([int(os.environ["RANK"]) + 1])
        dist.all_reduce(t)
        assert dist.get_world_size() == int(os.environ["WORLD_SIZE"]) == 3
        open(os.path.join({str(out)!r}, os.environ["RANK"]), "w").write(
            f"{{t.item()}} {{os.environ['LOCAL_RANK']}} {{sys.argv[1:]}}")
        dist.destroy_process_group()
        """)
    rc = bench.spawn_ranks(3, ["--gpus", "3"], script=s)
    assert rc == 0
    got = sorted(p.name for p in out.iterdir())
    assert got == ["0", "1", "2"]
    for r in range(3):
        total, lr, argv = (out / str(r)).read_text().split(" ", 2)
        assert total == "6" and lr == str(r) and "'--gpus', '3'" in argv


def test_spawn_ranks_first_failure_ends_the_job(tmp_path):
    s = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)  # a rank left waiting for its peer (a collective that never completes)
        """)
    t0 = time.monotonic()
    rc = bench.spawn_ranks(2, [], script=s)
    assert rc == 3
    assert time.monotonic() - t0 < 30


def test_bench_refuses_a_launcher_world_size_other_than_gpus():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE is 1" in r.stderr
    assert r.stdout == ""


def test_cpu_baseline_times_the_whole_partition(li001, monkeypatch):
    """bench.cpu_baseline over a whole partition: the box's CPU share of threads,
    the 1-thread point, and the count / Σ row id checked against the scan it is compared with."""
    from cubit_amd import filters as F
    from oracle import oracle as O

    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    cols = [O.Column(li001.l_shipdate), O.Column(li001.l_discount), O.Column(li001.l_quantity)]
    plan = F.serialize(F.q6_filter_set())
    ref = O.table_scan(cols, plan, li001.n_rows)
    k = 20_000
    sample = (cols, plan, k, None)
    full = (cols, plan, li001.n_rows, None)
    out = bench.cpu_baseline(sample, full, gpu=(len(ref), int(ref.sum())), min_seconds=0.3)
    assert out["equals_gpu_count_and_rowid_sum"] is True
    assert out["cores"] == min(3, out["host_cpus"]["affinity"])
    assert str(li001.n_rows) in out["sample"] and out["sample"].startswith("the whole partition")
    assert out["value"] > 0 and out["single_thread_value"] > 0
    bad = bench.cpu_baseline(sample, full, gpu=(len(ref) + 1, int(ref.sum())), min_seconds=0.1)
    assert bad["equals_gpu_count_and_rowid_sum"] is False
