"""bench.py's multi-GPU launcher and the step-roofline arithmetic, on the CPU.

`python bench.py --gpus N` (the driver's command) starts N ranks itself when no torchrun
environment is present; `--cpu-dry-run` rehearses that path on gloo (launcher, process group,
Trainer start-up broadcast, the per-step flat gradient all-reduce of the real model) without HIP.
"""
import json
import pathlib
import subprocess
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_starts_n_ranks(n):
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--cpu-dry-run", "--steps", "2", "--warmup", "1"],
                       cwd=ROOT, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == n and d["ranks_reported"] == list(range(n))
    assert d["config"]["parallelism"] == f"dp{n}" and d["config"]["backend"] == "gloo"
    assert d["allreduce_ok"] and d["params_broadcast_ok"]
    # the bucket holds every gradient + the BN running buffers + the non-finite flag
    assert d["allreduce_elems"] > 7_518_102


def test_bench_rejects_world_mismatch():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "PATH": "/usr/bin:/bin"}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu-dry-run"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode != 0 and "process group has 1 ranks" in (r.stderr + r.stdout)


def test_op_cost_matches_kernel_formulas():
    """roofline.step sums op_cost over the step's C-ABI ops: spot-check it against DESIGN.md §3."""
    from ogv.functional import op_cost, probe_bytes
    u = dict(M=1000, N=64, K=48, elem=2, res=True, bias=True)
    assert op_cost("gemm_fwd", u) == (probe_bytes("gemm_fwd", u), 2 * 1000 * 64 * 48)
    # MBConv at C = 48, mid = 192: forward passes x->e, e->d, d (pool), d->p, (p, x)->out
    b, f = op_cost("mbconv_fwd", dict(M=100, B=1, C=48, mid=192, se=12, elem=2))
    assert b == 2 * 100 * (48 + 192 + 2 * 192 + 192 + 192 + 48 + 3 * 48) + 4 * (2 * 192 * 48 + 9 * 192 + 2 * 192 * 12)
    assert f == 4 * 100 * 192 * 48 + 18 * 100 * 192
    b, _ = op_cost("layernorm_bwd", dict(M=10, C=8, elem=4, dres=True))
    assert b == 4 * 10 * 8 * 4 + 80 + 64
