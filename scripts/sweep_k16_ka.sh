#!/bin/bash
# Karatsuba threshold/leaf sweep for the K = 16 u32 multiply prefix (configs[3], d = dp = tau = 128)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export N=1024 KS=16 OPTS=${OPTS:-256:256,224:224,256:224,320:256,512:256,256:256}
timeout -k 10 500 python3 -u scripts/mul_rate.py
