"""Per-dispatch rocprofv3 counter summary of the LAST n dispatches of each kernel whose name contains a filter
(tools/layer_bench.py --only OP runs a full training step first; its timed reps are the last dispatches).
usage: python tools/pmc_last.py CSV [--match conv_pipe] [--last 5]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="conv_pipe")
    ap.add_argument("--last", type=int, default=5)
    args = ap.parse_args()
    for path in args.csv:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in csv.DictReader(open(path)):
            if args.match not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            per[d]["_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            names[d] = r["Kernel_Name"]
        by = collections.defaultdict(list)
        for d in sorted(per):
            by[names[d]].append(d)
        for k, ds in by.items():
            sel = ds[-args.last:]
            avg = {c: sum(per[d][c] for d in sel) / len(sel) for c in per[sel[0]]}
            print(f"{path}: {k[:110]} ({len(sel)} of {len(ds)} dispatches)")
            for c in sorted(avg):
                print(f"    {c:40s} {avg[c]:.5g}")


if __name__ == "__main__":
    main()
