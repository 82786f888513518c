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


def test_defaults_are_one_gpu_config2(bench, monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.config, a.dist_backend) == (1, 2, "nccl")
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
