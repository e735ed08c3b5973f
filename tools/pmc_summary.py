"""Summarise rocprofv3 --pmc passes (tools/pmc_conv.sh) for the conv kernels of one layer.

For each kernel family (conv_gemm fwd / dgrad, wgrad3, wgrad1) the LAST `n` dispatches of every pass
(the layer_bench repetitions) are averaged per counter, and the stall picture is derived:
SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES, MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 4 SIMDs x 256 CUs) when both are in one pass is
not available: the MFMA share is reported against SQ_BUSY_CYCLES instead).
usage: python tools/pmc_summary.py gpurun_out/pmc [n=3]
"""
import collections
import csv
import glob
import re
import sys


def family(name):
    n = name.replace("ym::(anonymous namespace)::", "").replace("void ", "")
    if "conv_gemm" in n:
        targs = [t.strip() for t in n.split("<")[1].split(">")[0].split(",")]
        return f"conv_gemm<{','.join(targs[:6])}> " + ("fwd" if targs[6] == "0" else "dgrad")
    return re.sub(r"[(<].*", "", n)


def main():
    root = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    vals = collections.defaultdict(dict)
    for path in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
        rows = list(csv.DictReader(open(path)))
        per = collections.defaultdict(lambda: collections.defaultdict(list))   # fam -> dispatch -> rows
        for r in rows:
            fam = family(r["Kernel_Name"])
            if not any(k in fam for k in ("conv_gemm", "wgrad3", "wgrad1", "conv_halo", "conv_pipe", "conv_hpipe")):
                continue
            per[fam][int(r["Dispatch_Id"])].append(r)
        for fam, disp in per.items():
            last = sorted(disp)[-n:]
            acc = collections.defaultdict(list)
            for d in last:
                for r in disp[d]:
                    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
            for c, v in acc.items():
                vals[fam][c] = sum(v) / len(v)
    for fam, c in vals.items():
        print(fam)
        wc = c.get("SQ_WAVE_CYCLES")
        for k in sorted(c):
            extra = ""
            if wc and k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                            "SQ_ACTIVE_INST_VMEM"):
                extra = f"  ({100 * c[k] / wc:.1f} % of wave cycles)"
            print(f"   {k:40s} {c[k]:16.0f}{extra}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "SQ_BUSY_CYCLES" in c:
            print(f"   MFMA busy / SQ busy: {c['SQ_VALU_MFMA_BUSY_CYCLES'] / c['SQ_BUSY_CYCLES']:.3f}")


if __name__ == "__main__":
    main()
