"""HBM traffic of every conv layer's fwd / dgrad / wgrad kernels, and of the dense 3x3 family per
training step, from two rocprofv3 counter passes over tools/layer_bench.py --seq-out.

usage: python tools/pmc_layers.py FETCH_counter_collection.csv WRITE_counter_collection.csv seq.json [SOURCE] [COMMIT]

layer_bench replays each layer's launches (reps + 2 per kind) in isolation and launches one torch
elementwise kernel after each group (three in a row before the first): the dispatches between two
markers are one group.  traffic = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section: on
gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads; rocprofv3 reports KB).
Per-launch bytes = group bytes / launches.  Writes profiles/traffic.json["family conv3x3 bs<B>"]
(bytes per training step: every k=3 layer's fwd + dgrad + wgrad once) and prints a per-layer table
with traffic / algorithmic bytes.
"""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def dispatches(path, counter):
    rows = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        d = int(r["Dispatch_Id"])
        ent = rows.setdefault(d, [r["Kernel_Name"], 0.0])
        ent[1] += float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def groups(disp, ngroups):
    """Counter sums of the last `ngroups` groups: each group ENDS with one separator, so the groups are the
    runs between the last ngroups + 1 separators (the warm-up training step before them launches torch
    elementwise kernels of its own, three in a row among them, so the start is anchored at the end)."""
    sep = [i for i, (n, _) in enumerate(disp) if "elementwise" in n]
    bounds = sep[-(ngroups + 1):]
    assert len(bounds) == ngroups + 1, (len(sep), ngroups)
    return [sum(v for _, v in disp[a + 1:b]) for a, b in zip(bounds[:-1], bounds[1:])]


def main():
    fetch_csv, write_csv, seq_json = sys.argv[1:4]
    source = sys.argv[4] if len(sys.argv) > 4 else str(Path(fetch_csv).parent)
    commit = sys.argv[5] if len(sys.argv) > 5 else None
    seq = json.loads(Path(seq_json).read_text())
    B = seq["batch"]
    G = seq["groups"]
    fetch = groups(dispatches(fetch_csv, "FETCH_SIZE"), len(G))
    write = groups(dispatches(write_csv, "WRITE_SIZE"), len(G))
    assert len(fetch) >= len(G) and len(write) >= len(G), (len(fetch), len(write), len(G))
    fam = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    alg3 = 0.0
    print(f"{'op':>4} {'kind':>6} k {'cin':>4} {'cout':>4} {'out':>7} {'MB/launch':>10} {'alg MB':>8} {'x alg':>6}")
    for g, f, w in zip(G, fetch, write):
        byts = (2 * f + w) * 1024 / g["launches"]
        oh, ow = g["out"]
        ih, iw = oh * g["s"], ow * g["s"]
        xin, yout, wb = B * ih * iw * g["cin"] * 2, B * oh * ow * g["cout"] * 2, g["cout"] * g["cin"] * g["k"] ** 2 * 2
        alg = xin + yout + wb
        print(f"{g['op']:4d} {g['kind']:>6} {g['k']} {g['cin']:4d} {g['cout']:4d} {oh:3d}x{ow:<3d} {byts / 1e6:10.1f} "
              f"{alg / 1e6:8.1f} {byts / alg:6.2f}")
        if g["k"] == 3:
            fam[g["kind"]] += byts
            alg3 += alg
    tot = sum(fam.values())
    print(f"3x3 family per step: {tot / 1e9:.2f} GB ({', '.join(f'{k} {v / 1e9:.2f}' for k, v in fam.items())}); "
          f"algorithmic {alg3 / 1e9:.2f} GB -> {tot / alg3:.2f}x")
    p = ROOT / "profiles" / "traffic.json"
    d = json.loads(p.read_text()) if p.exists() else {}
    d[f"family conv3x3 bs{B}"] = {"bytes_per_launch": int(tot), "unit": "bytes per training step",
                                  "by_direction": {k: int(v) for k, v in fam.items()},
                                  "algorithmic_bytes": int(alg3),
                                  "method": "tools/layer_bench.py --seq-out under two rocprofv3 --pmc passes "
                                            "(FETCH_SIZE, WRITE_SIZE), each layer's launches replayed in isolation",
                                  "source": source, "commit": commit}
    p.write_text(json.dumps(d, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
