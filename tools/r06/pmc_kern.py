"""Sum rocprofv3 --pmc counters per kernel name over a run's dispatches (counter_collection.csv), print per kernel:
dispatches, each counter's per-dispatch mean.  usage: python tools/r06/pmc_kern.py DIR [filter substring]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

d = Path(sys.argv[1])
filt = sys.argv[2] if len(sys.argv) > 2 else ""
f = next(d.rglob("*counter_collection.csv"))
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for row in csv.DictReader(open(f)):
    k = row["Kernel_Name"]
    if filt not in k:
        continue
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    disp[k].add(row["Dispatch_Id"])
for k, c in acc.items():
    n = len(disp[k])
    short = k.replace("void ym::(anonymous namespace)::", "").split("(ym::")[0][:110]
    print(f"{short}  [{n} dispatches]")
    for name in sorted(c):
        print(f"    {name:28s} {c[name] / n:14.4g}")
    m = c.get("SQ_INSTS_MFMA")
    if m:
        print(f"    per MFMA: SALU {c['SQ_INSTS_SALU'] / m:.2f}  VALU {c['SQ_INSTS_VALU'] / m:.2f}  LDS {c['SQ_INSTS_LDS'] / m:.2f}"
              "")
    if "SQ_WAVE_CYCLES" in c:
        print(f"    wait-any {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}  wait-inst {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}"
              f"  active {c['SQ_ACTIVE_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}  (fractions of wave cycles)")
