"""Summarise a rocprofv3 kernel trace stored as a rocpd SQLite database (rocprofv3's default output here).

Per kernel name: launches, total and average duration.  With --iter-kernel NAME (a kernel launched once per
iteration, e.g. the first kernel of a forward), also the per-iteration wall span (first start to last end of the
iteration's kernels), the summed kernel time and the time no kernel was running, averaged over the last --last
iterations.

usage: python tools/rocpd_summary.py DB [--iter-kernel prep_weights_kernel --last 20 --top 30 --sequence]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--iter-kernel", default=None)
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--sequence", action="store_true", help="also list the last iteration's kernels in order")
    args = ap.parse_args()
    db = sqlite3.connect(args.db)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    cnt, tot = collections.Counter(), collections.defaultdict(float)
    for n, s, e in rows:
        cnt[n] += 1
        tot[n] += (e - s) / 1e3
    print(f"{len(rows)} kernel dispatches")
    for n, t in sorted(tot.items(), key=lambda x: -x[1])[:args.top]:
        print(f"{t:10.1f} us {cnt[n]:6d} x {t / cnt[n]:7.2f} us  {n[:110]}")
    if args.iter_kernel:
        starts = [i for i, (n, _, _) in enumerate(rows) if args.iter_kernel in n]
        its = list(zip(starts, starts[1:] + [len(rows)]))[-args.last:]
        spans, busy, idle, nk = [], [], [], []
        for a, b in its:
            seg = rows[a:b]
            t0, t1 = seg[0][1], max(e for _, _, e in seg)
            ivs = sorted((s, e) for _, s, e in seg)
            cover, cur_s, cur_e = 0, ivs[0][0], ivs[0][1]
            for s, e in ivs[1:]:
                if s > cur_e:
                    cover += cur_e - cur_s
                    cur_s, cur_e = s, e
                else:
                    cur_e = max(cur_e, e)
            cover += cur_e - cur_s
            spans.append((t1 - t0) / 1e3)
            busy.append(sum(e - s for _, s, e in seg) / 1e3)
            idle.append((t1 - t0 - cover) / 1e3)
            nk.append(len(seg))
        k = len(its)
        if args.sequence:
            seg = rows[its[-1][0]:its[-1][1]]
            prev = seg[0][1]
            print("start_us  gap_us  dur_us  kernel (last iteration)")
            for n, s_, e_ in seg:
                print(f"{(s_ - seg[0][1]) / 1e3:8.1f} {(s_ - prev) / 1e3:7.1f} {(e_ - s_) / 1e3:7.2f}  {n[:100]}")
                prev = max(prev, e_)
        print(f"per iteration (last {k}): {sum(nk) / k:.0f} kernels, span {sum(spans) / k:.1f} us, "
              f"summed kernel time {sum(busy) / k:.1f} us, no kernel running {sum(idle) / k:.1f} us")


if __name__ == "__main__":
    main()
