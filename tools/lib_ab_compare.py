"""Compare per-layer timings of two library builds from tools/lib_ab_layers.sh (lb_A1, lb_B1, lb_A2, lb_B2):
mean of the two rounds per (op, direction), B vs A, and the summed change per direction.
usage: python tools/lib_ab_compare.py DIR"""
import glob
import os
import sys


def parse(path):
    rows = {}
    for ln in open(path):
        parts = ln.split("|")
        if len(parts) < 4 or not parts[0].strip()[:1].isdigit():
            continue
        op = int(parts[0].split()[0])
        geo = " ".join(parts[0].split()[1:6])
        t = [float(parts[i].split()[0]) for i in (1, 2, 3)]
        names = [p.strip() for p in parts[4:7]] if len(parts) >= 7 else ["", "", ""]
        rows[op] = (geo, t, names)
    return rows


def main(d):
    runs = {v: [parse(f) for f in sorted(glob.glob(os.path.join(d, f"lb_{v}*.txt")))] for v in "AB"}
    tot = {v: [0.0, 0.0, 0.0] for v in "AB"}
    for op in sorted(runs["A"][0]):
        geo, _, names = runs["B"][0][op]
        for k, kind in enumerate(("fwd", "dgrad", "wgrad")):
            ta = sum(r[op][1][k] for r in runs["A"]) / len(runs["A"])
            tb = sum(r[op][1][k] for r in runs["B"]) / len(runs["B"])
            tot["A"][k] += ta
            tot["B"][k] += tb
            if ta > 0 and abs(tb - ta) / ta > 0.02:
                print(f"op {op:3d} {geo:22s} {kind:5s} A {ta * 1e3:7.1f} us  B {tb * 1e3:7.1f} us ({100 * (tb / ta - 1):+5.1f} %)  "
                      f"{names[k]}")
    for k, kind in enumerate(("fwd", "dgrad", "wgrad")):
        print(f"{kind:5s} total: A {tot['A'][k]:.3f} ms  B {tot['B'][k]:.3f} ms ({100 * (tot['B'][k] / tot['A'][k] - 1):+.1f} %)")


if __name__ == "__main__":
    main(sys.argv[1])
