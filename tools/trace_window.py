"""Kernels of one training step inside a time window, in start order with their stream, duration and the GPU-idle gap
before each (no kernel running on any stream) — for reading where the step's idle gaps sit.

Steps are delimited by prep_weights_kernel (the middle step is shown); times in ms from that step's start.
usage: python tools/trace_window.py <run_kernel_trace.csv> <from_ms> <to_ms>
"""
import csv
import re
import sys


def short(name):
    n = name.replace("ym::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)[:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    lo, hi = float(sys.argv[2]), float(sys.argv[3])
    qkey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[qkey]) for r in rows)
    starts = [i for i, k in enumerate(ks) if "prep_weights" in k[2]]
    mid = len(starts) // 2
    seg = ks[starts[mid]:starts[mid + 1]]
    t0 = seg[0][0]
    busy_until = t0
    print(f"{'start':>8s} {'idle':>6s} {'dur':>7s}  stream  kernel")
    for s, e, n, q in seg:
        idle = max(0, s - busy_until)
        if lo <= (s - t0) / 1e6 <= hi:
            print(f"{(s - t0) / 1e6:8.3f} {idle / 1e3:6.1f} {(e - s) / 1e3:7.1f}  {q:>6s}  {short(n)}")
        busy_until = max(busy_until, e)


if __name__ == "__main__":
    main()
