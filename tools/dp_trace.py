"""When the bucket all-reduces go out against the backward's kernels, from a rocprofv3 kernel trace of the
data-parallel rehearsal (tools/dp_trace.sh: bench.py --gpus 2 over gloo, both ranks on GPU 0, YM_DP_MARK=1).

With YM_DP_MARK=1 yolomi/dist.py launches one tiny marker kernel (torch's spin_kernel, torch.cuda._sleep) on the bucket's comm
stream right before each bucket's collective, after the comm stream's waits on the events of the launches that
wrote the bucket.  A marker's START is therefore the moment the bucket's collective could begin.  For the last
backward of each rank this prints every marker's start relative to the backward's first kernel and the number
of backward kernels that started after it (buckets overlapping the backward have many).
usage: python tools/dp_trace.py <rocprofv3 output dir>
"""
import csv
import glob
import os
import sys


def main(root):
    for kf in sorted(glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)):
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "?"))
                    for r in csv.DictReader(open(kf)))
        lb = [s for s, e, n, q in ks if "loss_bwd" in n]
        opt = [s for s, e, n, q in ks if "grad_sqnorm" in n]
        if not lb or not opt:
            continue
        b0 = lb[-1]
        b1 = min(s for s in opt if s > b0)
        marks = [(s, q) for s, e, n, q in ks if "spin_kernel" in n and b0 <= s < b1]
        bk = [(s, e, n) for s, e, n, q in ks if b0 <= s < b1 and "spin_kernel" not in n]
        if not bk:
            continue
        last = max(e for s, e, n in bk)
        print(f"{os.path.basename(kf)}: last backward {len(bk)} kernels over {(last - b0) / 1e6:.2f} ms, "
              f"{len(marks)} bucket markers")
        for s, q in marks:
            after = sum(1 for s2, e2, n2 in bk if s2 > s)
            print(f"  bucket marker (stream {q}) at {(s - b0) / 1e6:7.3f} ms: {after:4d} of {len(bk)} backward kernels "
                  f"start later")


if __name__ == "__main__":
    main(sys.argv[1])
