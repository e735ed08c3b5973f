"""Per-kernel-family dynamic instruction mix from a rocprofv3 --pmc CSV (tools/r05/insts.sh): summed over all
dispatches of each kernel template, instructions per MFMA (or per wave where a kernel has no MFMA) and time."""
import collections
import csv
import re
import sys


def family(name):
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        f = family(r["Kernel_Name"])
        d = r["Dispatch_Id"]
        agg[f][r["Counter_Name"]] += float(r["Counter_Value"])
        if d not in seen[f]:
            seen[f].add(d)
            agg[f]["_us"] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["_us"])
    print(f"{'kernel':70s} {'n':>4s} {'us':>9s} {'MFMA':>9s} {'SALU/M':>7s} {'VALU/M':>7s} {'LDS/M':>6s} {'VMEM/M':>7s}")
    for f, c in rows:
        if c["_us"] < 50:
            continue
        m = c.get("SQ_INSTS_MFMA", 0)
        den = m if m > 0 else max(c.get("SQ_WAVES", 1), 1)
        print(f"{f[:70]:70s} {len(seen[f]):4d} {c['_us']:9.1f} {m:9.3g} {c.get('SQ_INSTS_SALU', 0) / den:7.2f} "
              f"{c.get('SQ_INSTS_VALU', 0) / den:7.2f} {c.get('SQ_INSTS_LDS', 0) / den:6.2f} "
              f"{(c.get('SQ_INSTS_VMEM_RD', 0) + c.get('SQ_INSTS_VMEM_WR', 0)) / den:7.2f}{'' if m > 0 else '  (per wave)'}")


if __name__ == "__main__":
    main(sys.argv[1])
