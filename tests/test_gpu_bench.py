"""bench.py on the GPU: the measurement contract of every line, and the multi-rank path with the
real engine.

  - every `secondary` line of the default bench carries a `roofline` and a `cpu_baseline` (the
    oracle's 1-thread rate, measured or labelled extrapolated), and the lines that verify their
    results report them correct;
  - `bench.py --gpus 2 --workload mixed` with the gloo backend (two ranks sharing the one GPU of a
    test box: the rehearsal mode of bench.setup_dist, never the measured configuration) runs the
    engine on both ranks: rank 1 loads the keys rank 0 broadcast (bench.make_context), each rank
    runs its shard of configs[4] through the strong-scaling chunk loop, the decrypted results are
    gathered, and every sum and product is correct.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(args, env=None, timeout=280):
    e = dict(os.environ, **(env or {}))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=e,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.strip().splitlines() if ln.startswith("{")]
    assert lines, p.stdout[-2000:]
    return json.loads(lines[-1])


def test_bench_every_line_has_roofline_and_cpu_baseline():
    d = _run_bench(["--steps", "4", "--warmup", "2", "--cpu-seconds", "3"])
    assert d["roofline"]["frac"] > 0 and d["cpu_baseline"]["value"] > 0
    sec = d["secondary"]
    assert "error" not in sec, sec.get("error")
    for name in ("u32_encrypt_decrypt", "u32_encrypt", "u32_decrypt_fresh", "u32_decrypt_after_add",
                 "u32_add_pcie_inclusive", "u8_mul", "u8_decrypt_after_mul", "u32_mul_low12",
                 "u32_mul_low16", "u32_mul_low16_batch16384", "u32_mul_low20", "u32_mul_low24_batch2",
                 "u32_mul_full_extrapolated", "mixed_config4",
                 "config0_u8_encrypt", "config0_u8_decrypt", "config0_u8_add"):
        line = sec[name]
        assert line["value"] > 0, name
        r = line["roofline"]
        assert r["bound"] in ("hbm", "mfma", "pcie") and r["peak"] > 0 and r["achieved"] > 0, name
        assert (r["bound"] == "pcie") == (name == "u32_add_pcie_inclusive"), name
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-9, name
        assert r["frac"] <= 1.0, (name, r["frac"])  # issued work, never an algorithm's count
        c = line["cpu_baseline"]
        assert c["value"] > 0 and c["cores"] == 1 and c["kind"] == "port", name
    assert sec["u8_mul"]["verified"] and sec["u8_decrypt_after_mul"]["verified"]
    assert sec["config0_u8_decrypt"]["verified"]
    assert sec["config0_u8_add"]["verified"]["correct_sums"] == sec["config0_u8_add"]["batch"]
    assert sec["u32_mul_low16"]["cpu_baseline"]["extrapolated"] is True
    # configs[3] names batch 1024; the batch-16384 rate is a labelled aside
    assert sec["u32_mul_low12"]["batch"] == sec["u32_mul_low16"]["batch"] == 1024
    assert sec["u32_mul_low20"]["batch"] == 1024  # result bits 16..19 at configs[3]'s batch
    assert sec["u32_mul_low16_batch16384"]["batch"] == 16384
    assert sec["u32_mul_low20_batch16"]["batch"] == 16
    assert sec["u32_mul_low24_batch2"]["batch"] == 2  # result bits 20..23 (split plans)
    assert sec["u32_mul_low12"]["cpu_baseline"].get("extrapolated") is None
    m = sec["mixed_config4"]
    assert m["verified"]["correct_sums"] == m["verified"]["correct_products"] == m["global_batch"]


def test_bench_two_ranks_run_the_engine():
    n = 262144
    d = _run_bench(["--gpus", "2", "--workload", "mixed", "--batch", str(n), "--steps", "1",
                    "--warmup", "1"], env={"HM_BENCH_BACKEND": "gloo"})
    assert d["world_size_seen"] == 2 and d["n_gpus"] == 2
    assert d["config"]["batch_per_gpu"] == n // 2
    assert d["verified"] == {"correct_sums": n, "correct_products": n, "of": n}


def test_bench_two_ranks_headline_add():
    """The headline add path (run_add) at world size 2 on one card (gloo): each rank adds its own
    4096-value shard (weak scaling), the sustained-clock replays run per rank, and rank 0 gathers
    every sum for the check (the driver's N-GPU runs take this path over RCCL)."""
    d = _run_bench(["--gpus", "2", "--steps", "3", "--warmup", "1"], env={"HM_BENCH_BACKEND": "gloo"})
    assert d["world_size_seen"] == 2 and d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 8192 and d["verified"]["of"] == 8192
    assert d["verified"]["correct_sums"] >= 8192 - 16  # (the scheme's noise aside)
    assert d["roofline"]["sustained"]["kernel_ms"] > 0
