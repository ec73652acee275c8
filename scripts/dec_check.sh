#!/bin/bash
# Decrypt/encrypt kernels: the -m gpu tests that decrypt, then the bench's cipher secondary lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/dec; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "enc or dec or add or mul_parity or golden or kat or wire" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/dec/bench.json").read().strip().splitlines()[-1])
for k in ("u32_decrypt_after_add", "u32_decrypt_fresh", "u32_encrypt", "u32_encrypt_decrypt"):
    s = d["secondary"][k]
    print(k, s["value"], s["kernel_us_per_step"], s["roofline"]["frac"], s.get("predrawn_masks", ""))
print("headline ms", d["ms_per_step"])
PY
