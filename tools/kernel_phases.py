#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of one default `bench.py` run into its two
timed phases (tools/final_profile.sh):
  pipelined  warmup + steps launches with renders in flight: per-dispatch
             durations overlap, so the amortized time per launch is the span
             of the timed dispatches (first start -> last end) / steps;
  serial     warmup + steps launches one at a time: the average dispatch
             duration is the kernel's own time, which bench.py's
             roofline.kernel_ms measures with HIP events.
  python tools/kernel_phases.py TRACE.csv KERNEL_SUBSTR STEPS WARMUP [OUT.json [BENCH.log]]
BENCH.log: the profiled bench run's own output; its JSON line's ms_per_step (the
pipelined step as that run timed it, profiler included) is reported beside the
trace's amortized span per launch, which it should match."""
import csv
import json
import sys


def main():
    path, kname, steps, warmup = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if kname in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = warmup + steps
    if len(rows) < 2 * n:
        sys.exit(f"{len(rows)} {kname} dispatches, expected >= {2 * n}")
    pipe, ser = rows[-2 * n:-n][warmup:], rows[-n:][warmup:]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # noqa: E731
    span = (max(int(r["End_Timestamp"]) for r in pipe) - min(int(r["Start_Timestamp"]) for r in pipe)) / 1e6
    out = {"kernel": rows[0]["Kernel_Name"], "steps": steps, "warmup": warmup,
           "serial_avg_dispatch_ms": sum(dur(r) for r in ser) / len(ser),
           "pipelined_avg_dispatch_ms": sum(dur(r) for r in pipe) / len(pipe),
           "pipelined_span_per_launch_ms": span / len(pipe),
           "note": "serial = one launch at a time (bench.py roofline.kernel_ms); pipelined dispatches overlap, "
                   "so their per-dispatch durations include their neighbours' time: the amortized time per "
                   "launch is the span of the timed dispatches / steps"}
    if len(sys.argv) > 6:
        for line in open(sys.argv[6]):
            if line.startswith("{"):
                b = json.loads(line)
                out["profiled_run_ms_per_step"] = b["ms_per_step"]
                out["profiled_run_kernel_ms"] = b["roofline"]["kernel_ms"]
                out["span_per_launch_over_step"] = out["pipelined_span_per_launch_ms"] / b["ms_per_step"]
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 5:
        json.dump(out, open(sys.argv[5], "w"), indent=1)


if __name__ == "__main__":
    main()
