"""bench.py --gpus N without torchrun launches its own N ranks (VERDICT r03
item 3): the launcher (distributed.launch_ranks) and bench.py's rank-0 line
assembly, exercised with a gloo stand-in worker on CPU."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

WORKER = os.path.join(HERE, "_rank_worker.py")


def _env():
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e["OMP_NUM_THREADS"] = "1"
    return e


def test_launch_ranks_gloo_world2():
    from gibbssampler_amd.distributed import launch_ranks
    line, out = launch_ranks(2, WORKER, ["--gpus", "2"], env=_env(), timeout=240)
    assert line["n_gpus"] == 2
    assert line["ranks_seen"] == [0, 1]
    assert line["value"] == 2.0                    # the max over ranks


def test_launch_ranks_failure_raises():
    from gibbssampler_amd.distributed import launch_ranks
    with pytest.raises(RuntimeError):
        launch_ranks(2, os.path.join(HERE, "does_not_exist.py"), [], env=_env(), timeout=240)


def test_bench_self_launch_line():
    """python bench.py --gpus 2 (no torchrun): the parent spawns 2 ranks and prints
    rank 0's line with n_gpus == --gpus; the ranks get --no-cpu-baseline."""
    e = _env()
    e["GS_BENCH_RANK_SCRIPT"] = WORKER
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "centered",
                          "--no-cpu-baseline"], env=e, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["gpus_arg"] == 2
    assert "--no-cpu-baseline" in line["argv"]


def test_bench_world_mismatch_exits_nonzero():
    """WORLD_SIZE set but different from --gpus: refuse instead of measuring."""
    e = _env()
    e.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu-baseline"],
                         env=e, cwd=ROOT, capture_output=True, text=True, timeout=120)
    assert out.returncode == 2


def test_attach_cpu_assembly():
    import bench
    line = {"metric": "m", "n_gpus": 2, "cpu_baseline": None, "pcg": {"cg_iterations_per_solve": 100.0}}
    cpu = {"value": 0.5, "unit": "chain-iterations/s", "cores": 16, "kind": "port", "sample": "x {n_cg}",
           "seconds_per_iteration": 2.0, "pcg_parts": {"t_rhs": 1.0, "t_cg": 0.01, "t_rest": 0.0, "n_sampled": 10}}
    out = bench.attach_cpu(dict(line), cpu)
    assert out["cpu_baseline"]["value"] == pytest.approx(1.0 / (1.0 + 100 * 0.01), rel=1e-5)
    assert "100.0" in out["cpu_baseline"]["sample"]
    ready = {"value": 3.0, "unit": "chain-iterations/s", "cores": 16, "kind": "port", "sample": "s"}
    assert bench.attach_cpu(dict(line), ready)["cpu_baseline"] == ready


def test_bench_parse_defaults(monkeypatch):
    """bench.py's defaults: the driver's 20-step command samples 5 sweeps for the
    roofline timing (every 4th), long runs every 10th; --opt pairs are kept for
    the line's config (library options set before any plan is made)."""
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--steps", "20", "--warmup", "5"])
    a = bench.parse()
    assert (a.steps, a.warmup, a.time_every, a.nchains) == (20, 5, 4, 32)
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.steps, a.time_every) == (500, 10)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "masked_asis", "--opt", "GS_SHT_MERGE_RINGS=0"])
    a = bench.parse()
    assert (a.nchains, a.lmax, a.nside, a.steps) == (1, 512, 256, 5)
    assert a.opt == ["GS_SHT_MERGE_RINGS=0"]
