"""GPU busy vs idle time per training step from a rocprofv3 kernel trace.

Steps are delimited by the prep_weights_kernel launch (one per forward).  For each step:
wall (first kernel start -> next step's first kernel start), busy (union of kernel intervals over
all streams) and the largest idle gaps with the kernels on either side.
usage: python tools/trace_gaps.py <run_kernel_trace.csv> [top=8]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    starts = [i for i, k in enumerate(ks) if "prep_weights" in k[2]]
    for a, b in zip(starts, starts[1:]):
        seg = ks[a:b]
        wall = ks[b][0] - seg[0][0]
        busy, cur_s, cur_e = 0, seg[0][0], seg[0][1]
        gaps = []
        prev_name = seg[0][2]
        for s, e, n in seg[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, prev_name[:60], n[:60]))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev_name = n if e >= cur_e else prev_name
        busy += cur_e - cur_s
        print(f"step: wall {wall / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(wall - busy) / 1e6:.3f} ms  "
              f"kernels {len(seg)}  gaps {len(gaps)}")
        for g, p, n in sorted(gaps, reverse=True)[:top]:
            print(f"   {g / 1e3:8.1f} us  after {p}  before {n}")


if __name__ == "__main__":
    main()
