"""Per-step kernel breakdown from a rocprofv3 --kernel-trace CSV (eager bench run): the dispatches
between the last two AdamW launches form one train step; prints them grouped by kernel instance +
grid, with time and share."""
import collections
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    m = re.match(r"^(?:void )?(\w+)(<[^>]*>)?", n)
    if n.startswith("_ZN12_GLOBAL__N_1"):
        m2 = re.match(r"_ZN12_GLOBAL__N_1\d+(\w+?)I(.*)E", n)
        return (m2.group(1) + "<" + m2.group(2)[:40] + ">") if m2 else n[:60]
    return (m.group(1) + (m.group(2) or "")) if m else n[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    a, b = ad[-2] + 1, ad[-1] + 1
    step = rows[a:b]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
    print(f"one step: {len(step)} dispatches, wall {(t1 - t0) / 1e3:.1f} us, kernel-busy {busy / 1e3:.1f} us")
    g = collections.OrderedDict()
    for r in step:
        k = (short(r["Kernel_Name"]), r["Grid_Size_X"], r["Workgroup_Size_X"])
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        g.setdefault(k, []).append(d)
    tot = sorted(g.items(), key=lambda kv: -sum(kv[1]))
    for (name, grid, wg), ds in tot[: int(sys.argv[2]) if len(sys.argv) > 2 else 60]:
        print(f"{sum(ds) / 1e3:9.1f} us {100 * sum(ds) / busy:5.1f}%  n={len(ds):3d} avg {sum(ds) / len(ds) / 1e3:8.1f} us  "
              f"grid={int(grid) // int(wg):6d}x{wg:4s} {name}")


if __name__ == "__main__":
    main()
