"""Minimal HIP-graph capture patterns with several streams (debugging the 3-stream capture crash).

Each case captures a few elementwise torch kernels under torch.cuda.graph with side streams joined by
events, then replays once.  usage: python tools/hip_graph_repro.py CASE   (cases: see CASES)
"""
import sys

import torch

dev = torch.device("cuda", 0)
x = torch.zeros(1 << 20, device=dev)
EVS = []          # events recorded during a capture stay alive until the process ends


def fork_join(streams, body):
    main = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(main)
    EVS.append(ev)
    for s in streams:
        s.wait_event(ev)
    body(main)
    for s in streams:
        e = torch.cuda.Event()
        e.record(s)
        main.wait_event(e)
        EVS.append(e)


def case_two(main, s1, s2):            # main <-> s1 only (s2 joined, idle)
    with torch.cuda.stream(s1):
        x.add_(1)
    e = torch.cuda.Event()
    e.record(s1)
    EVS.append(e)
    main.wait_event(e)
    x.add_(1)


def case_idle_third(main, s1, s2):     # s2 joined but never used, s1 works
    with torch.cuda.stream(s1):
        x.add_(1)


def case_reuse_event(main, s1, s2):    # one event re-recorded on two streams
    e = torch.cuda.Event()
    EVS.append(e)
    with torch.cuda.stream(s1):
        x.add_(1)
    e.record(s1)
    s2.wait_event(e)
    with torch.cuda.stream(s2):
        x.add_(1)
    e.record(s2)
    main.wait_event(e)


def case_side_to_side(main, s1, s2):   # s2 waits on an event recorded on s1 (neither is the origin)
    with torch.cuda.stream(s1):
        x.add_(1)
    e = torch.cuda.Event()
    e.record(s1)
    EVS.append(e)
    s2.wait_event(e)
    with torch.cuda.stream(s2):
        x.add_(1)


# the stream / event pattern of the first 46 forward ops of the n@256 plan at 3 scheduler streams
# (tools/graph_debug.py prefix 46): (stream, ops whose events it waits for, records its own event)
SCHED46 = [[0, [], False]] * 12 + [[0, [], True]] + [[0, [], False]] * 4 + [[0, [], True]] + [
    [1, [12], False], [1, [17], False], [1, [12], False], [1, [], False], [1, [], True], [1, [], False],
    [1, [], False], [1, [], False], [1, [], False], [1, [], True], [2, [22], False], [2, [27], False],
    [2, [22], False], [2, [], False], [2, [], False], [2, [], False], [2, [], True], [2, [], True],
    [2, [], False], [2, [], False], [2, [], False], [2, [], False], [2, [], False], [2, [], True],
    [0, [35], False], [0, [41], True], [1, [34], False], [1, [43], False]]
OP_EVS = {}


def run_sched(main, s1, s2, n):
    streams = [main, s1, s2]
    for i, (k, waits, rec) in enumerate(SCHED46[:n]):
        for j in waits:
            streams[k].wait_event(OP_EVS[j])
        with torch.cuda.stream(streams[k]):
            x.add_(1)
        if rec:
            ev = OP_EVS.setdefault(i, torch.cuda.Event())
            ev.record(streams[k])


def run_sched_latest(main, s1, s2, n):
    """As run_sched, but every wait goes to the NEWEST event recorded so far on the producer's stream."""
    streams = [main, s1, s2]
    last = {}
    for i, (k, waits, rec) in enumerate(SCHED46[:n]):
        for j in waits:
            src = SCHED46[j][0]
            streams[k].wait_event(OP_EVS[last[src]])
        with torch.cuda.stream(streams[k]):
            x.add_(1)
        if rec:
            ev = OP_EVS.setdefault(i, torch.cuda.Event())
            ev.record(streams[k])
            last[k] = i


def case_sched46_latest(main, s1, s2):
    run_sched_latest(main, s1, s2, 46)


def case_older_wait(main, s1, s2):     # s1 waits on an event s2 recorded BEFORE its latest one
    ea, eb = torch.cuda.Event(), torch.cuda.Event()
    EVS.extend([ea, eb])
    with torch.cuda.stream(s2):
        x.add_(1)
    ea.record(s2)
    with torch.cuda.stream(s2):
        x.add_(1)
    eb.record(s2)
    main.wait_event(eb)
    s1.wait_event(ea)
    with torch.cuda.stream(s1):
        x.add_(1)


RELAY = {}


def run_sched_relay(main, s1, s2, n):
    """As run_sched, but a wait between two non-origin streams goes through the origin stream: the
    producer's event is waited by main, which records a relay event the consumer waits for."""
    streams = [main, s1, s2]
    for i, (k, waits, rec) in enumerate(SCHED46[:n]):
        for j in waits:
            src = SCHED46[j][0]
            if k != 0 and src != 0:
                main.wait_event(OP_EVS[j])
                r = RELAY.setdefault(k, torch.cuda.Event())
                r.record(main)
                streams[k].wait_event(r)
            else:
                streams[k].wait_event(OP_EVS[j])
        with torch.cuda.stream(streams[k]):
            x.add_(1)
        if rec:
            ev = OP_EVS.setdefault(i, torch.cuda.Event())
            ev.record(streams[k])


def case_sched46_relay(main, s1, s2):
    run_sched_relay(main, s1, s2, 46)


def case_cycle(main, s1, s2):          # s2 waits on s1, later s1 waits on s2 (both non-origin)
    ea, eb = torch.cuda.Event(), torch.cuda.Event()
    EVS.extend([ea, eb])
    with torch.cuda.stream(s1):
        x.add_(1)
    ea.record(s1)
    s2.wait_event(ea)
    with torch.cuda.stream(s2):
        x.add_(1)
    eb.record(s2)
    s1.wait_event(eb)
    with torch.cuda.stream(s1):
        x.add_(1)


def case_sched44(main, s1, s2):
    run_sched(main, s1, s2, 44)


def case_sched46(main, s1, s2):
    run_sched(main, s1, s2, 46)


CASES = {"sched44": case_sched44, "sched46": case_sched46, "sched46_latest": case_sched46_latest,
         "older_wait": case_older_wait, "sched46_relay": case_sched46_relay, "cycle": case_cycle, "two": case_two, "idle_third": case_idle_third, "reuse_event": case_reuse_event,
         "side_to_side": case_side_to_side}

if __name__ == "__main__":
    name = sys.argv[1]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    fn = CASES[name]
    fork_join([s1, s2], lambda m: fn(m, s1, s2))       # eager once
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    mode = sys.argv[2] if len(sys.argv) > 2 else "global"
    with torch.cuda.graph(g, capture_error_mode=mode):
        fork_join([s1, s2], lambda m: fn(m, s1, s2))
    g.replay()
    torch.cuda.synchronize()
    print(name, "captured and replayed", float(x[0]), flush=True)
