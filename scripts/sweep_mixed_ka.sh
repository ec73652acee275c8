#!/bin/bash
# Karatsuba threshold/leaf sweep for configs[4]'s multiply half (K = 8 at d = dp = tau = 256, one
# 131,072-value launch chunk); scripts/mul_rate.py prints ms per batch and checks identical bits.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export N=131072 KS=8 PARAMS=256,256,1,256 OPTS=${OPTS:-192:192,128:128,160:160,256:192,256:256,0:256}
timeout -k 10 500 python3 -u scripts/mul_rate.py
