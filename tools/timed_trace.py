#!/usr/bin/env python3
"""The bench's two timers against the kernel trace.

bench.py reports, for the dominant kernel, (a) `ms_per_step`: HIP events around the whole timed region
/ K (every launch and the gaps between them), and (b) `kernel_ms`: the library's HIP events recorded
around each launch, in a separate pass of K more steps after the timed region.  rocprofv3's
`--kernel-trace` gives every launch's own start / end.  This tool takes a trace of a bench command and the
bench's JSON line (from the same run), finds the K timed launches (after the settle and warmup steps) and
the K launches of the events pass, and prints their per-launch durations next to (a) and (b):

    python tools/timed_trace.py <run_kernel_trace.csv> <bench log or json> [kernel substring] [--out f.json]

One step must be one launch of the named kernel (c2 / c3 / c5 / c6: the plain encode / decode)."""
import csv
import json
import statistics
import sys


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--out")]
    out = None
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
        args = [x for x in args if x != out]
    trace, log = args[0], args[1]
    kname = args[2] if len(args) > 2 else "encode16_kernel"
    line = [ln for ln in open(log).read().splitlines() if ln.strip().startswith("{")][-1]
    b = json.loads(line)
    S, W, K = b["settle_steps"], b["warmup"], b["steps"]
    rows = [r for r in csv.DictReader(open(trace)) if kname in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    n = len(rows)
    if n < S + W + 2 * K:
        raise SystemExit(f"{n} launches of {kname}, expected >= {S + W + 2 * K} (settle {S} + warmup {W} + 2 x {K})")
    # the timed launches: the K after settle + warmup (any launches before the settle, e.g. the encode
    # feeding a decode bench, come first: count from the end of the trace's runs of this kernel)
    t0 = n - 2 * K
    timed = range(t0, t0 + K)
    evpass = range(t0 + K, t0 + 2 * K)
    dur = [(en[i] - st[i]) / 1e6 for i in timed]
    gaps = [(st[i + 1] - en[i]) / 1e6 for i in timed if i + 1 < t0 + K]
    span = (en[t0 + K - 1] - st[t0]) / 1e6
    dur_ev = [(en[i] - st[i]) / 1e6 for i in evpass]
    gaps_ev = [(st[i + 1] - en[i]) / 1e6 for i in evpass if i + 1 < t0 + 2 * K]
    r = {
        "kernel": kname, "launches_in_trace": n, "settle_steps": S, "warmup": W, "steps": K,
        "timed_launch_ms": [round(x, 5) for x in dur],
        "timed_mean_ms": statistics.mean(dur), "timed_median_ms": statistics.median(dur),
        "timed_min_ms": min(dur), "timed_max_ms": max(dur),
        "timed_gap_mean_ms": statistics.mean(gaps) if gaps else None,
        "timed_span_first_start_to_last_end_ms": span,
        "bench_ms_per_step": b["ms_per_step"],
        "bench_device_region_ms_per_step": b["roofline"].get("device_ms_per_step"),
        "events_pass_launch_ms_mean": statistics.mean(dur_ev),
        "events_pass_gap_mean_ms": statistics.mean(gaps_ev) if gaps_ev else None,
        "bench_kernel_ms_events": b["roofline"].get("kernel_ms"),
        "all_launches_mean_ms": statistics.mean((e - s) / 1e6 for s, e in zip(st, en)),
    }
    r["span_per_step_ms"] = span / K
    r["event_minus_trace_ms"] = (r["bench_kernel_ms_events"] or 0) - r["events_pass_launch_ms_mean"]
    print(json.dumps(r, indent=1))
    if out:
        json.dump(r, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
