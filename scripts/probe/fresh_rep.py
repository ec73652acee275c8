"""Repeats test_unseeded_keys_and_masks_are_fresh's body N times on the selected library."""
import sys, numpy as np
sys.path.insert(0, "homomorph-rust_amd")
import homomorph as H
bad = 0
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    p = H.Parameters(128, 128, 1, 128)
    c1 = H.Context(p)
    c1.generate_secret_key(); c1.generate_public_key()
    x = np.arange(64, dtype=np.uint32)
    for _ in range(4):
        e = c1.encrypt(x)
        d = c1.decrypt(e)
        if not np.array_equal(d, x):
            bad += 1
            print("mismatch", it, np.nonzero(d != x)[0][:8], d[:8])
print("bad", bad)
