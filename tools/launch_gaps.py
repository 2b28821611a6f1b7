"""Launch gaps from a rocprofv3 kernel trace: where the GPU sits idle between consecutive dispatches.

    python tools/launch_gaps.py RUN_kernel_trace.csv [--match rmr_jit_trace] [--last N]

Sorts the dispatches by start time and, over the window from the first to the last dispatch whose name
contains --match (the trace kernel), reports the span, the busy time (union of the dispatch intervals),
and every gap end_i -> start_{i+1} grouped by the pair of kernel kinds around it (trace, fold, fill =
hipMemsetAsync's rocclr kernel, copy, other). `--last N`: only the last N trace dispatches' window (the
timed region of a bench run comes after its warm-up). Used for bench.py --api render (the reference's
call pattern: one small launch per tile and sample) and the launch-bound configs."""
import argparse
import csv
import json
import statistics


def kind(name):
    n = name.lower()
    if "rmr_jit_trace" in n or "k_trace" in n:
        return "trace"
    if "fold" in n:
        return "fold"
    if "fill" in n:
        return "fill"
    if "copy" in n:
        return "copy"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="trace")
    ap.add_argument("--last", type=int, default=0)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    tr = [i for i, r in enumerate(rows) if kind(r[2]) == a.match]
    if not tr:
        raise SystemExit("no %s dispatches" % a.match)
    if a.last:
        tr = tr[-a.last:]
    # the window starts at the first dispatch after the previous trace (the call's own memset etc.)
    lo = tr[0]
    while lo > 0 and kind(rows[lo - 1][2]) in ("fill", "copy"):
        lo -= 1
    hi = tr[-1] + 1
    while hi < len(rows) and kind(rows[hi][2]) in ("fold",):
        hi += 1
    w = rows[lo:hi]
    span = w[-1][1] - w[0][0]
    busy, cur_s, cur_e = 0, w[0][0], w[0][1]
    for s, e, _ in w[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    gaps = {}
    for (s0, e0, n0), (s1, e1, n1) in zip(w, w[1:]):
        gaps.setdefault("%s->%s" % (kind(n0), kind(n1)), []).append((s1 - e0) / 1e3)
    dur = {}
    for s, e, n in w:
        dur.setdefault(kind(n), []).append((e - s) / 1e3)
    calls = len(tr)
    out = {"trace_dispatches": calls, "span_ms": round(span / 1e6, 4), "busy_ms": round(busy / 1e6, 4),
           "idle_ms": round((span - busy) / 1e6, 4), "idle_us_per_trace": round((span - busy) / 1e3 / calls, 3),
           "us_per_trace_dispatch": round(span / 1e3 / calls, 3),
           "durations_us": {k: {"n": len(v), "mean": round(statistics.mean(v), 3), "median": round(statistics.median(v), 3)}
                            for k, v in sorted(dur.items())},
           "gaps_us": {k: {"n": len(v), "mean": round(statistics.mean(v), 3), "median": round(statistics.median(v), 3),
                           "max": round(max(v), 3)} for k, v in sorted(gaps.items())}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
