"""Per-launch-class view of a scripts/pmc_cmd.sh directory: the MFMA-carrying kernels grouped by
(kernel, grid size) -- the multiplier's schoolbook launches share one kernel name, and their size
class shows in the grid -- with launches, time per launch (kernel trace), matrix-core busy (the
SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES ratio scaled so that the 25-chunk chain reads as its
GRBM-normalised 0.75) and non-MFMA VALU instructions per MFMA.
usage: python3 scripts/pmc_classes.py DIR [norm]"""
import collections
import csv
import os
import sys

root = sys.argv[1]
norm = float(sys.argv[2]) if len(sys.argv) > 2 else 32.2


def per_dispatch(path):
    d, meta = collections.defaultdict(dict), {}
    for r in csv.DictReader(open(path)):
        k = r["Dispatch_Id"]
        d[k][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[k] = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))
    return d, meta


sq, meta = per_dispatch(os.path.join(root, "sq", "run_counter_collection.csv"))
dur = collections.defaultdict(list)
for r in csv.DictReader(open(os.path.join(root, "trace", "run_kernel_trace.csv"))):
    dur[r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"])].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
grp = collections.defaultdict(list)
for k, c in sq.items():
    if c.get("SQ_INSTS_MFMA", 0) > 0:
        grp[meta[k]].append(c)
print(f"{'kernel':44s} {'grid':>10s} {'n':>4s} {'ms/launch':>9s} {'busy':>5s} {'valu/mfma':>9s}")
for key in sorted(grp, key=lambda k: (k[0], k[1])):
    L = grp[key]
    mf = sum(c["SQ_INSTS_MFMA"] for c in L)
    va = sum(c["SQ_INSTS_VALU"] for c in L)
    busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"] for c in L) / sum(c["SQ_BUSY_CYCLES"] for c in L) / norm
    t = dur.get(key, [0.0])
    print(f"{key[0][-44:]:44s} {key[1]:10d} {len(L):4d} {sum(t) / len(t):9.3f} {busy:5.2f} {(va - mf) / mf:9.2f}")
