"""bench.py's driver contract on the CPU (no GPU): defaults, the cpu_baseline leg
on a tiny sample, and the committed PMC traffic it reports next to the roofline."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    import bench as b
    return b


def test_defaults_are_one_gpu_config3(bench, monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.config, a.dist_backend) == (1, 3, "nccl")
    assert a.steps > 0 and a.warmup > 0 and a.cpu_seconds > 0
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "7", "--warmup", "2"])
    a = bench.parse()
    assert (a.gpus, a.steps, a.warmup) == (8, 7, 2)


@pytest.mark.parametrize("cfgid", [2, 3, 4])
def test_cpu_baseline_leg(bench, cfgid):
    """The CPU codec on a bounded sample of the same workload, as bench reports it."""
    from fecgpu import workloads
    cfg = workloads.CONFIGS[cfgid]
    out = bench.cpu_baseline(cfg, 0.05, 2)
    assert set(out) >= {"value", "unit", "cores", "kind", "sample"}
    assert out["unit"] == "GB/s" and out["cores"] == 2 and out["kind"] == "port"
    assert out["value"] > 0 and cfg.name in out["sample"]


def test_cpu_baseline_leg_sliding_window(bench):
    """Config 7 (sliding-window RLC): the vectorised, threaded CPU codec on the
    config's stream shape (here a shortened stream)."""
    from fecgpu import workloads
    cfg = workloads.CONFIGS[7]
    out = bench.cpu_baseline_sw(cfg, 0.05, 2, nsrc=16384)
    assert out["unit"] == "GB/s" and out["cores"] == 2 and out["kind"] == "port"
    assert out["value"] > 0 and "16384 sources" in out["sample"] and "simd" in out["codec"]


@pytest.mark.parametrize("cfgid,kernel", [(2, "encode"), (2, "decode"), (3, "encode"), (3, "decode"),
                                          (4, "encode"), (4, "decode")])
def test_committed_pmc_traffic(bench, cfgid, kernel):
    """The HBM traffic bench puts in roofline.traffic comes from the committed
    rocprofv3 FETCH_SIZE / WRITE_SIZE summary of that config."""
    t, src = bench.pmc_traffic(cfgid, kernel)
    assert t is not None and src.startswith("profiles/r") and src.endswith(f"_cfg{cfgid}_traffic.json")
    d = json.load(open(os.path.join(ROOT, src)))
    k = d["kernels"][kernel]
    assert k["traffic_bytes"] == k["read_bytes"] + k["write_bytes"] == t


def test_cfg2_traffic_close_to_algorithmic(bench):
    """cfg2 encode moves (k + r) * S bytes per window: 65,536 x 10 x 1,200 B; the
    measured HBM traffic is within a few percent of it (no wasted re-reads)."""
    t, _ = bench.pmc_traffic(2, "encode")
    alg = 65536 * 10 * 1200
    assert 1.0 <= t / alg < 1.1


def test_gpus_flag_launches_n_ranks(bench):
    """`python bench.py --gpus N` (the driver's form, no launcher) must
    run N ranks, one per GPU.  On this GPU-less host the ranks stop at the first
    device call, but both must have started with WORLD_SIZE = 2."""
    import subprocess
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "1", "--dist-backend", "gloo", "--cpu-seconds", "0"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert "launching 2 ranks" in r.stderr
    assert "rank 0/2" in r.stderr and "rank 1/2" in r.stderr, r.stderr[-3000:]
    # no GPU here: both ranks join the gloo group, then leave cleanly (exit 2, which the launcher reports as a failure), never
    # one rank torn down by the launcher before the other has started
    assert r.stderr.count("no GPU visible") == 2 and r.returncode != 0, r.stderr[-3000:]


def test_gpus_flag_refuses_without_enough_gpus(bench):
    """RCCL runs one rank per GPU: --gpus 4 with fewer visible GPUs is an error,
    not a run on GPU 0 labelled n_gpus 4."""
    import subprocess
    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 2 and "needs 4 GPUs" in r.stderr


def test_world_size_must_match_gpus(bench):
    import subprocess
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 2 and "refusing" in r.stderr


def test_host_share_bounds_threads(bench, monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.host_share() == min(3, len(os.sched_getaffinity(0)))
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.host_share() == len(os.sched_getaffinity(0))
