"""Multi-stream timeline of one train step from a rocprofv3 --kernel-trace CSV (default bench run:
eager launches, encoder prefetch stream, weight-gradient side stream). The step is the span
between two consecutive AdamW launches in the middle of the run. Prints wall, the union of busy intervals (any kernel
running), the summed kernel time per stream, the share of wall with 0 / 1 / >=2 kernels in
flight, and the kernels that run ALONE longest (the critical-path candidates).

    python tools/timeline.py run_kernel_trace.csv [top]
"""
import collections
import csv
import sys

from trace_step import short


def main(path, top=25):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    k = len(ad) // 2  # a step inside the timed region (the tail holds bench.py's probe replays)
    t0 = int(rows[ad[k - 1]]["End_Timestamp"])
    t1 = int(rows[ad[k]]["End_Timestamp"])
    step = [r for r in rows if int(r["End_Timestamp"]) > t0 and int(r["Start_Timestamp"]) < t1]
    ev = []
    for r in step:
        a, b = max(int(r["Start_Timestamp"]), t0), min(int(r["End_Timestamp"]), t1)
        ev.append((a, 1, r))
        ev.append((b, -1, r))
    ev.sort(key=lambda e: (e[0], e[1]))
    depth, last = 0, t0
    hist = collections.Counter()
    alone = collections.Counter()
    running = set()
    for t, d, r in ev:
        hist[min(depth, 2)] += t - last
        if depth == 1 and running:
            (only,) = running
            alone[running_names[only]] += t - last
        last = t
        depth += d
        if d > 0:
            running.add(r["Kernel_Name"] + r["Dispatch_Id"])
            running_names[r["Kernel_Name"] + r["Dispatch_Id"]] = short(r["Kernel_Name"])
        else:
            running.discard(r["Kernel_Name"] + r["Dispatch_Id"])
    hist[min(depth, 2)] += t1 - last
    wall = t1 - t0
    per_stream = collections.Counter()
    for r in step:
        per_stream[r["Queue_Id"]] += min(int(r["End_Timestamp"]), t1) - max(int(r["Start_Timestamp"]), t0)
    print(f"step wall {wall / 1e3:.1f} us, {len(step)} dispatches")
    print(f"  idle {hist[0] / 1e3:.1f} us ({100 * hist[0] / wall:.1f}%), one kernel {hist[1] / 1e3:.1f} us "
          f"({100 * hist[1] / wall:.1f}%), >=2 kernels {hist[2] / 1e3:.1f} us ({100 * hist[2] / wall:.1f}%)")
    for q, t in sorted(per_stream.items()):
        print(f"  queue {q}: kernel time {t / 1e3:.1f} us")
    print("kernels running alone (us):")
    for name, t in alone.most_common(top):
        print(f"  {t / 1e3:8.1f}  {name[:90]}")


running_names = {}

if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
