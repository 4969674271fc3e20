"""Per-step accounting of a rocprofv3 kernel-trace CSV of a replayed step (tools/decoder_trace.py or bench.py):
the step = dispatches between the last two AdamW launches; per queue its kernel-busy time and the idle gaps
between its consecutive kernels (the launch / drain latency a dependent chain pays), and the kernel families
by total time. Usage: python tools/trace_gaps.py kernel_trace.csv"""
import collections
import csv
import sys

from step_timeline import short


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    a, b = ad[-2] + 1, ad[-1] + 1
    step = rows[a:b]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    print(f"step: {len(step)} dispatches, wall {(t1 - t0) / 1e3:.1f} us")
    qkey = "Queue_Id" if "Queue_Id" in step[0] else "Stream_Id"
    byq = collections.defaultdict(list)
    for r in step:
        byq[r[qkey]].append(r)
    for q, rs in sorted(byq.items()):
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
        gaps = [max(0, int(y["Start_Timestamp"]) - int(x["End_Timestamp"])) for x, y in zip(rs, rs[1:])]
        gs = sorted(gaps)
        med = gs[len(gs) // 2] if gs else 0
        print(f"  queue {q}: {len(rs)} kernels, busy {busy / 1e3:.1f} us, gaps {sum(gaps) / 1e3:.1f} us "
              f"(median {med / 1e3:.2f} us, {sum(1 for g in gaps if g > 5000)} over 5 us)")
    fam = collections.Counter()
    cnt = collections.Counter()
    for r in step:
        k = short(r["Kernel_Name"])
        fam[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        cnt[k] += 1
    print("kernel families (us per step, launches, us per launch):")
    for k, v in fam.most_common(30):
        print(f"  {v / 1e3:8.1f} {cnt[k]:4d} {v / 1e3 / cnt[k]:7.1f}  {k}")


if __name__ == "__main__":
    main()
