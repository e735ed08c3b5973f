"""Per-stream view of one training step from a rocprofv3 kernel trace: where the step's wall time
goes and which stream holds the tail.

Steps are delimited by prep_weights_kernel (one per forward).  For the middle step: per stream
(queue) busy time, first start / last end relative to the step start, the forward / backward split
(first loss kernel), and the kernel families ranked by time on the critical (last-finishing) path.
usage: python tools/trace_streams.py <run_kernel_trace.csv>
"""
import collections
import csv
import re
import sys


def family(name):
    n = name.replace("ym::(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return re.sub(r"<.*", "", n)


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    qkey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[qkey]) for r in rows)
    starts = [i for i, k in enumerate(ks) if "prep_weights" in k[2]]
    if len(starts) < 3:
        print("need >= 3 steps in the trace")
        return
    mid = len(starts) // 2
    seg = ks[starts[mid]:starts[mid + 1]]
    t0 = seg[0][0]
    wall = ks[starts[mid + 1]][0] - t0
    loss0 = next((s for s, e, n, q in seg if "loss" in n or "assign" in n), None)
    print(f"step wall {wall / 1e6:.3f} ms; forward ends at {(loss0 - t0) / 1e6 if loss0 else float('nan'):.3f} ms")
    per_q = collections.defaultdict(list)
    for s, e, n, q in seg:
        per_q[q].append((s, e, n))
    for q, L in sorted(per_q.items(), key=lambda kv: kv[1][0][0]):
        busy = sum(e - s for s, e, _ in L)
        fams = collections.Counter()
        for s, e, n in L:
            fams[family(n)] += e - s
        top = ", ".join(f"{k} {v / 1e6:.2f}" for k, v in fams.most_common(5))
        print(f"stream {q}: {len(L)} kernels, busy {busy / 1e6:.3f} ms, span {(L[0][0] - t0) / 1e6:.3f} .. "
              f"{(L[-1][1] - t0) / 1e6:.3f} ms | {top}")
    # union busy and the step's tail: what runs after the last non-side kernel
    cur_s, cur_e, busy = seg[0][0], seg[0][1], 0
    for s, e, _, _ in seg[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"union busy {busy / 1e6:.3f} ms of {wall / 1e6:.3f} ({busy / wall:.1%})")
    # idle gaps (no kernel on any stream): where the wall time the union misses goes
    gaps, cur_e, prev = [], seg[0][1], seg[0]
    for k in seg[1:]:
        if k[0] > cur_e:
            gaps.append((k[0] - cur_e, cur_e - t0, prev[2], k[2]))
        if k[1] >= cur_e:
            cur_e, prev = k[1], k
    tail = ks[starts[mid + 1]][0] - cur_e
    big = sorted(gaps, reverse=True)
    hist = collections.Counter()
    for g, *_ in gaps:
        hist["<2us" if g < 2000 else "2-10us" if g < 10000 else "10-50us" if g < 50000 else ">=50us"] += g
    print(f"idle gaps: {len(gaps)}, {sum(g for g, *_ in gaps) / 1e6:.3f} ms (" +
          ", ".join(f"{k} {v / 1e6:.3f}" for k, v in sorted(hist.items())) + f"); after the last kernel {tail / 1e6:.3f} ms")
    for g, at, a, b in big[:12]:
        print(f"  gap {g / 1e3:7.1f} us at {at / 1e6:7.3f} ms  after {family(a)[:40]:40} before {family(b)[:40]}")
    if "--windows" in sys.argv:
        # the kernels of every stream around the largest gaps: what was the GPU waiting for
        for g, at, a, b in big[:6]:
            lo, hi = t0 + at - 60000, t0 + at + g + 60000
            print(f"-- window around the {g / 1e3:.1f}-us gap at {at / 1e6:.3f} ms")
            for s_, e_, n_, q_ in seg:
                if e_ >= lo and s_ <= hi:
                    print(f"   q{q_} {(s_ - t0) / 1e6:8.3f} .. {(e_ - t0) / 1e6:8.3f}  {family(n_)[:60]}")
    last = sorted(seg, key=lambda k: k[1])[-25:]
    print("last kernels to finish:")
    for s, e, n, q in last:
        print(f"  q{q} {(s - t0) / 1e6:8.3f} .. {(e - t0) / 1e6:8.3f}  {family(n)[:70]}")


if __name__ == "__main__":
    main()
