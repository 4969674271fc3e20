"""Concurrency timeline of ONE train step from a rocprofv3 --kernel-trace CSV (eager bench run; the
step = the end of one AdamW to the end of the next, every dispatch overlapping it, clipped): wall, time with 0 / 1 / 2 / 3+ kernels in
flight, per-queue busy time, and per kernel family the time it ran ALONE (nothing else on the chip:
the critical-path suspects). Usage: python tools/step_timeline.py kernel_trace.csv"""
import collections
import csv
import re
import sys


def short(n):
    """Kernel family name: the function name and its template arguments, namespaces dropped."""
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("_ZN12_GLOBAL__N_1"):
        m = re.match(r"_ZN12_GLOBAL__N_1\d+(\w+?)I(.*)E", n)
        return (m.group(1) + "<" + m.group(2)[:40] + ">") if m else n[:60]
    m = re.match(r"^(?:void )?(\w+)(<[^>]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    # the shortest span between consecutive AdamW launches with no foreign kernel in it (bench.py's
    # roofline probe and the timing spin run after the timed steps)
    spans = [(int(rows[j]["End_Timestamp"]) - int(rows[i + 1]["Start_Timestamp"]), i + 1, j + 1)
             for i, j in zip(ad, ad[1:]) if not any("spin" in r["Kernel_Name"] for r in rows[i + 1:j + 1])]
    _, a, b = min(spans)
    # the step: from the end of one AdamW to the end of the next, with EVERY dispatch that overlaps that
    # interval (clipped to it) -- also the next step's kernels that start while the closing AdamW runs, which a
    # window by dispatch order would drop (it made AdamW look alone)
    t0, t1 = int(rows[a - 1]["End_Timestamp"]), int(rows[b - 1]["End_Timestamp"])
    step = [r for r in rows if int(r["Start_Timestamp"]) < t1 and int(r["End_Timestamp"]) > t0
            and "spin" not in r["Kernel_Name"]]
    ev = []
    for i, r in enumerate(step):
        ev.append((max(int(r["Start_Timestamp"]), t0), 1, i))
        ev.append((min(int(r["End_Timestamp"]), t1), -1, i))
    ev.sort()
    active = set()
    hist = collections.Counter()
    alone = collections.Counter()
    last = t0
    for t, kind, i in ev:
        dt = t - last
        if dt > 0:
            hist[min(len(active), 3)] += dt
            if len(active) == 1:
                (only,) = tuple(active)
                alone[short(step[only]["Kernel_Name"])] += dt
        last = t
        if kind == 1:
            active.add(i)
        else:
            active.discard(i)
    wall = t1 - t0
    qkey = "Queue_Id" if "Queue_Id" in step[0] else ("Stream_Id" if "Stream_Id" in step[0] else None)
    print(f"one step: {len(step)} dispatches, wall {wall / 1e3:.1f} us")
    print("  in flight: " + ", ".join(f"{k}{'+' if k == 3 else ''}: {hist[k] / 1e3:.1f} us ({100 * hist[k] / wall:.1f}%)"
                                      for k in range(4)))
    if qkey:
        q = collections.Counter()
        for r in step:
            q[r[qkey]] += min(int(r["End_Timestamp"]), t1) - max(int(r["Start_Timestamp"]), t0)
        for k, v in sorted(q.items()):
            print(f"  {qkey} {k}: kernel time {v / 1e3:.1f} us")
    print("ran alone (us):")
    for k, v in alone.most_common(25):
        print(f"  {v / 1e3:8.1f}  {k}")


if __name__ == "__main__":
    main()
