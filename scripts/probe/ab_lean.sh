set -u
KS=16 N=1024 bash scripts/ab_mulrate.sh k16lmin lmin129 lmin193 || exit 1
bash scripts/ab_mixed.sh lmin129 lmin193
