"""HBM traffic of the bench's probe kernel and of its kernel families, from two rocprofv3 counter passes.

usage: python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv bench.json [SOURCE]
Writes/updates profiles/traffic.json:
  [probe key]            bytes per launch of the probe conv (the bench's heaviest forward conv)
  ["family <k> bs<B>"]   bytes per training step of every launch of kernel family k
                         (fwd / dgrad / wgrad conv kernels, bn = the BatchNorm streaming + finalize kernels)

Counters (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE come from the L2's
memory-side request counters; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
coalesced reads — the conv kernels' staging (buffer_load dwordx4 ... lds) and the BN kernels'
16-B vector loads — so traffic = 2 x FETCH_SIZE + WRITE_SIZE.  rocprofv3 reports both in KB.
Steps in the pass = prep_weights_kernel dispatches (one per forward).
"""
import csv
import json
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def targs(name):
    m = re.search(r"<([^<>]*)>", name)
    return [t.strip() for t in m.group(1).split(",")] if m else []


def conv_kind(name):
    """'fwd' / 'dgrad' / 'wgrad' / None for a conv kernel dispatch name."""
    n = name.replace("ym::(anonymous namespace)::", "").replace("void ", "")
    t = targs(n)
    if n.startswith("conv_gemm_kernel<"):           # <BM,BN,WM,WN,KB,NS,MODE,ABL?>
        return "fwd" if t[6] == "0" else "dgrad"
    if n.startswith("conv_pipe_kernel<"):           # <BM,BN,WM,WN,MODE,ABL>
        return "fwd" if t[4] == "0" else "dgrad"
    if n.startswith("conv_halo_kernel<"):           # <...,MODE,ABL>
        return "fwd" if t[6] == "0" else "dgrad"
    if n.startswith("conv_direct_kernel<"):         # <NT,KC,KS,S,MODE,TP>
        return "fwd" if t[4] == "0" else "dgrad"
    if n.startswith("conv_direct_quad_kernel<"):    # stride-2 data gradient over 2x2-pixel quads
        return "dgrad"
    if n.startswith("conv_hpipe_kernel<"):          # <BN,WM,WN,MODE,WRES>
        return "fwd" if t[3] == "0" else "dgrad"
    if n.startswith(("wgrad3_kernel", "wgrad1_kernel", "wgrad_generic_kernel", "wgrad_reduce_kernel")):
        return "wgrad"
    if n.startswith(("bn_apply_kernel", "bn_bwd_reduce_kernel", "bn_bwd_apply_kernel", "bn_finalize_fused_kernel",
                     "stem_bwd_wgrad_kernel",
                     "partials_reduce_kernel", "bn_finalize_kernel", "bn_bwd_finalize_kernel")):
        return "bn"
    return None


def rows_of(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def main():
    fetch_csv, write_csv, bench_json = sys.argv[1:4]
    source = sys.argv[4] if len(sys.argv) > 4 else str(Path(fetch_csv).parent)
    b = json.loads(Path(bench_json).read_text().strip().splitlines()[-1])
    key, rank, per_step = b["probe"]["key"], b["probe"]["rank"], b["probe"]["count"]
    batch = b["config"]["batch_per_gpu"]
    probe, fam, steps = {}, {}, {}
    for counter, path in (("FETCH_SIZE", fetch_csv), ("WRITE_SIZE", write_csv)):
        rows = rows_of(path, counter)
        steps[counter] = sum(1 for r in rows if "prep_weights_kernel" in r["Kernel_Name"])
        # the probe: a step's forward conv launches in dispatch order (ConvBN 1, Detect level 2 each)
        fwd = [r for r in rows if conv_kind(r["Kernel_Name"]) == "fwd"]
        assert len(fwd) % per_step == 0, (len(fwd), per_step)
        sel = fwd[rank::per_step]
        names = {r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0] for r in sel}
        assert len(names) == 1, names
        probe[counter] = [float(r["Counter_Value"]) * 1024.0 for r in sel]
        for r in rows:
            k = conv_kind(r["Kernel_Name"])
            if k:
                fam.setdefault(k, {}).setdefault(counter, 0.0)
                fam[k][counter] += float(r["Counter_Value"]) * 1024.0
    n = min(len(probe["FETCH_SIZE"]), len(probe["WRITE_SIZE"]))
    fetch = sum(probe["FETCH_SIZE"][:n]) / n
    write = sum(probe["WRITE_SIZE"][:n]) / n
    f = ROOT / "profiles" / "traffic.json"
    d = json.loads(f.read_text()) if f.exists() else {}
    d[key] = {"bytes_per_launch": round(2 * fetch + write), "fetch_bytes_x2": round(2 * fetch),
              "write_bytes": round(write), "launches": n, "kernel": sorted(names)[0], "source": source}
    print(key, d[key])
    for k, v in sorted(fam.items()):
        fs, ws = v.get("FETCH_SIZE", 0.0) / steps["FETCH_SIZE"], v.get("WRITE_SIZE", 0.0) / steps["WRITE_SIZE"]
        d[f"family {k} bs{batch}"] = {"bytes_per_launch": round(2 * fs + ws), "unit": "bytes per training step",
                                      "fetch_bytes_x2": round(2 * fs), "write_bytes": round(ws),
                                      "steps": steps["FETCH_SIZE"], "source": source}
        print(f"family {k}", d[f"family {k} bs{batch}"])
    f.write_text(json.dumps(d, indent=1) + "\n")


if __name__ == "__main__":
    main()
