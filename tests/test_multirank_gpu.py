"""GPU: bench.py's multi-rank path end to end on a one-GPU box — two or four ranks (all on GPU 0, MAM_BENCH_ONE_DEVICE) with
the LBA write-back exchange over gloo (MAM_DIST_BACKEND) instead of RCCL, which refuses two ranks on one device. The
exchange blocks must have the same size on every rank (each rank's windows differ), the ranks' collectives must pair
up, and rank 0's in-run parity section must hold."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("cfg,ranks,extra", [("c3", 2, []), ("c2", 2, ["--batch", "128"]), ("c4", 4, [])])
def test_bench_ranks_one_gpu(cfg, ranks, extra):
    """c4: four of BASELINE configs[4]'s 8 agents' GPUs as four ranks (two agents each), neighbouring ranks' LBA
    windows overlapping (cross-rank write conflicts resolved in rank order)."""
    env = dict(os.environ, MAM_BENCH_ONE_DEVICE="1", MAM_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(ranks), "--config", cfg,
                        "--steps", "8", "--warmup", "2", "--no-cpu-baseline", "--no-latency", "--no-pose", "--no-sin",
                        *extra], capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.strip().splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == ranks and d["value"] > 0 and d.get("parity_ok"), d.get("invalid")
    p = d["parity"]
    assert p["extract_bit_exact"] and p["local_search_index_exact"] and p["triangulation_index_exact"]
    assert p["lba_same_control_flow"] and p["lba_max_point_rel_diff"] <= 1e-4
    assert d["lba"]["exchange_bytes_per_step"] > 0
