import re, sys, glob, collections
D = sys.argv[1]
runs = {}
for f in sorted(glob.glob(f"{D}/lb_*.txt")):
    name = f.split("lb_")[1][:-4]
    rows = {}
    for ln in open(f):
        parts = ln.split("|")
        if len(parts) < 7 or not parts[0].strip()[:1].isdigit():
            continue
        op = int(parts[0].split()[0])
        geo = " ".join(parts[0].split()[1:6])
        t = [float(parts[i].split()[0]) for i in (1, 2, 3)]
        k = [parts[i].strip() for i in (4, 5, 6)]
        rows[op] = (geo, t, k)
    runs[name] = rows
base = runs["default"]
gain = [0.0, 0.0, 0.0]
for op, (geo, t, k) in base.items():
    for d in range(3):
        best = min(((r[op][1][d], n, r[op][2][d]) for n, r in runs.items() if op in r and r[op][1][d] > 0), default=None)
        if best and best[0] < 0.97 * t[d] and t[d] - best[0] > 0.002:
            gain[d] += t[d] - best[0]
            print(f"op {op:3d} {geo:22s} {['fwd','dgrad','wgrad'][d]:5s} default {t[d]*1e3:6.1f} us [{k[d]}]  best {best[0]*1e3:6.1f} us [{best[2]}] ({best[1]})")
print("possible gain ms (fwd, dgrad, wgrad):", [round(g, 3) for g in gain])
