"""bench.py end to end on the GPU box, small frames: the one-GPU line and the
N-rank path that `bench.py --gpus N` launches by itself (on a one-GPU box the ranks
share the device and reduce through gloo, and the line says so)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _bench(*args, timeout=300):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_one_gpu_line():
    d = _bench("--gpus", "1", "--samples", "16", "--steps", "2", "--warmup", "1", "--no-cpu-baseline")
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["image_ok"]
    assert d["roofline"]["bound"] == "valu_fp64" and 0 < d["roofline"]["frac"] < 1
    assert d["roofline"]["kernel_ms_avg"] <= d["ms_per_step"]
    assert d["ptmi_trace_call"]["ms"] > 0


@pytest.mark.parametrize("config", ["c2", "c5"])
def test_bench_launches_ranks_itself(config):
    d = _bench("--gpus", "2", "--config", config, "--samples", "16", "--steps", "1", "--warmup", "1")
    assert d["n_gpus"] == 2 and d["image_ok"]
    assert len(d["per_rank"]["kernel_ms"]) == 2 and all(k > 0 for k in d["per_rank"]["kernel_ms"])
    assert d["cpu_baseline"] is None and d["ptmi_trace_call"] is None


def test_bench_extra_configs_line():
    """The other BASELINE configurations timed after the headline at the same GPU count
    (the default run does c3,c5; here at 2 ranks sharing the device, one timed frame each)."""
    d = _bench("--gpus", "2", "--samples", "16", "--steps", "1", "--warmup", "0", "--extra", "c3,c5",
               "--extra-steps", "1")
    assert d["config"]["scene"] == "reference" and d["n_gpus"] == 2
    ex = d["extra_configs"]
    assert sorted(ex) == ["c3", "c5"]
    assert ex["c3"]["config"]["split"] == "sample" and ex["c5"]["config"]["split"] == "tile"
    for v in ex.values():
        assert v["image_ok"] and v["value"] > 0 and len(v["per_rank_kernel_ms"]) == 2
        assert v["config"]["spp"] == 2048 and v["steps"] == 1
