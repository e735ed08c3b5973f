"""Cross-stream dependency latency on this GPU: the gap between a producer kernel's end and the start of a
consumer kernel on another stream that waits for it (hipStreamWaitEvent), vs the gap between two kernels
of one stream.  Run under `rocprofv3 --kernel-trace --output-format csv` and pass the trace to
`--analyze`:

  rocprofv3 --kernel-trace --output-format csv -d out -o run -- python3 tools/stream_wait_probe.py
  python3 tools/stream_wait_probe.py --analyze out/.../run_kernel_trace.csv

Cases (each repeated, separated by host syncs; the kernels are tiny elementwise adds tagged by size):
  same      A; B on one stream
  ready     s2 busy with a long spin while A runs on s1; s2 then waits on A's event (already complete) -> B
  parked    s2 idle, waits on A's event while s1 still spins before A -> B (the wait is pending when reached)
"""
import sys


def run():
    import torch
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    tag = {k: torch.zeros(n, device=dev) for k, n in (("A", 1001), ("B", 1002), ("C", 1003))}
    for _ in range(3):
        tag["A"].add_(1)
    torch.cuda.synchronize()
    for rep in range(20):
        # same stream
        with torch.cuda.stream(s1):
            torch.cuda._sleep(200000)
            tag["A"].add_(1)
            tag["B"].add_(1)
        torch.cuda.synchronize()
        # ready: the event completes while s2 is still busy
        ev = torch.cuda.Event()
        with torch.cuda.stream(s1):
            tag["A"].add_(1)
            ev.record(s1)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(400000)
            s2.wait_event(ev)
            tag["B"].add_(1)
        torch.cuda.synchronize()
        # parked: s2 reaches the wait long before the producer runs
        ev = torch.cuda.Event()
        with torch.cuda.stream(s1):
            torch.cuda._sleep(400000)
            tag["C"].add_(1)
            ev.record(s1)
        with torch.cuda.stream(s2):
            s2.wait_event(ev)
            tag["B"].add_(1)
        torch.cuda.synchronize()


def analyze(path):
    import csv
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
    ks = [k for k in ks if "elementwise" in k[2] or "spin" in k[2].lower() or "sleep" in k[2].lower()]
    ks = ks[next(i for i, k in enumerate(ks) if "spin" in k[2].lower() or "sleep" in k[2].lower()):]   # first case
    out = {"same": [], "ready": [], "parked": []}
    for i in range(0, len(ks) - 8, 9):
        w = ks[i:i + 9]
        out["same"].append(w[2][0] - w[1][1])
        r = sorted(w[3:6], key=lambda k: k[0])
        out["ready"].append(r[2][0] - max(r[0][1], r[1][1]))
        out["parked"].append(w[8][0] - w[7][1])
    for k, v in out.items():
        v = sorted(v)
        if v:
            print(f"{k:7s} n={len(v):3d}  median {v[len(v) // 2] / 1e3:7.1f} us  min {v[0] / 1e3:7.1f}  max {v[-1] / 1e3:7.1f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
