"""Summarise a rocprofv3 kernel_stats.csv per kernel family, per training step.
usage: python tools/prof_summary.py <run_kernel_stats.csv> [steps=7]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
fam = collections.defaultdict(lambda: [0.0, 0])
for r in rows:
    n = r["Name"]
    k = re.sub(r"\(.*", "", n.replace("ym::(anonymous namespace)::", "").replace("void ", ""))
    if "conv_gemm" in n:
        targs = [t.strip() for t in n.split("<")[1].split(">")[0].split(",")]
        k = "conv_gemm " + ("fwd" if targs[6] == "0" else "dgrad")   # <BM,BN,WM,WN,KB,NS,MODE,ABL>
    else:
        k = re.sub(r"<.*", "", k)
    fam[k][0] += float(r["TotalDurationNs"]) / 1e6 / steps
    fam[k][1] += int(r["Calls"]) // steps
tot = sum(v[0] for v in fam.values())
print(f"total kernel time {tot:.3f} ms/step")
for k, (t, c) in sorted(fam.items(), key=lambda x: -x[1][0])[:30]:
    print(f"{t:7.3f} ms {100 * t / tot:5.1f}% {c:5d} calls  {k}")
