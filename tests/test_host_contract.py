"""CPU tests of host-side contracts: key byte I/O, the mask CSPRNG restatement, the bench's
multi-rank entry, and the C ABI's host-only entry points.  No GPU."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import chacha20_block

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chacha20_known_answer():
    """The all-zero key / nonce block of Bernstein's ChaCha20 (the published test vector)."""
    blk = chacha20_block([0] * 8, 0, 0)
    assert blk[:16].hex() == "76b8e0ada0f13d90405d6ae55386bd28"
    assert blk[48:].hex() == "6a43b8f41518a11cc387b669b2ee6586"


def test_secret_key_bytes_round_trip():
    """context.rs:616-624: SecretKey::from_bytes(&[5, 14, 8]) -> to_bytes -> from_bytes."""
    import homomorph as H
    sk = H.SecretKey.from_bytes(bytes([5, 14, 8]))
    assert sk.limbs.tolist() == [5 | 14 << 8 | 8 << 16]       # polynomial.rs:108-122, LE limbs
    b = sk.to_bytes()
    assert len(b) == 8                                         # every limb, 8 bytes each (:99-105)
    assert H.SecretKey.from_bytes(b) == sk
    with pytest.raises(ValueError):
        H.SecretKey.from_bytes(b"")                            # "must not be empty" (:109)


def test_public_key_bytes_round_trip():
    """context.rs:626-635: PublicKey::from_bytes(&[[4,7,5],[1,2,3],[5,4,6]]) round trip."""
    import homomorph as H
    rows = [bytes([4, 7, 5]), bytes([1, 2, 3]), bytes([5, 4, 6])]
    pk = H.PublicKey.from_bytes(rows)
    assert pk.limbs.shape == (3, 1)
    assert pk.limbs[:, 0].tolist() == [4 | 7 << 8 | 5 << 16, 1 | 2 << 8 | 3 << 16, 5 | 4 << 8 | 6 << 16]
    assert H.PublicKey.from_bytes(pk.to_bytes()) == pk


def test_polynomial_byte_conversion():
    """polynomial.rs:606-612: trailing zero limbs survive to_bytes and compare equal."""
    import homomorph as H
    limbs = np.array([0b1001, 0b1000_0011_0101_1010, 0, 1, 0], dtype=np.uint64)
    sk = H.SecretKey(limbs)
    assert len(sk.to_bytes()) == 40
    assert H.SecretKey.from_bytes(sk.to_bytes()) == sk


def _bench(*args, env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                          capture_output=True, text=True, timeout=240, env=e)


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` starts two ranks itself (no external launcher); rank 0 reports the
    world size torch.distributed saw, the gathered shards and rank 0's broadcast keys."""
    r2 = _bench("--gpus", "2", "--workload", "distcheck")
    assert r2.returncode == 0, r2.stderr[-2000:]
    line2 = json.loads([l for l in r2.stdout.splitlines() if l.startswith("{")][-1])
    assert line2["n_gpus"] == 2 and line2["world_size_seen"] == 2
    assert line2["gathered_ok"] and line2["value"] == 128
    r1 = _bench("--gpus", "1", "--workload", "distcheck")
    line1 = json.loads([l for l in r1.stdout.splitlines() if l.startswith("{")][-1])
    assert line1["key_digest"] == line2["key_digest"]  # every rank got rank 0's keys


def test_bench_rejects_world_size_mismatch():
    r = _bench("--gpus", "4", "--workload", "distcheck",
               env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)
