"""Condense rocprofv3 rocpd databases (tools/profile_round.sh) into the summaries committed under
profiles/ (the --stats tables themselves, run_kernel_stats.csv, are copied there as they are):

  <prefix>_pmc.json          per-kernel FETCH_SIZE / WRITE_SIZE averages (separate passes) and the
                             HBM bytes per launch with the gfx950 correction of
                             MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of 16-B/lane
                             streaming reads -> x2; WRITE_SIZE exact for 16-B stores; both in KiB)

    python tools/rocpd_summary.py --trace D/trace/run_results.db --fetch D/fetch/run_results.db \
        --write D/write/run_results.db --out profiles/r01
"""
import argparse
import json
import re
import sqlite3


def short(name: str) -> str:
    """Demangled kernel names carry long parameter lists; keep the template head."""
    n = re.sub(r"^void ", "", name)
    n = n.replace("(anonymous namespace)::", "")
    m = re.match(r"^_ZN12_GLOBAL__N_1\d+(\w+?)I", n)
    if m:
        return m.group(1)
    return n.split("(")[0] if not n.startswith("(") else n


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    return [(short(r[0]), r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4])) for r in rows]


def pmc(db, counter):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, count(*), avg(value), avg(duration) from counters_collection "
                     "where counter_name = ? group by kernel_name", (counter,)).fetchall()
    return {short(r[0]): {"launches": int(r[1]), "avg_kib": float(r[2]), "avg_ns": float(r[3])} for r in rows}


def sq_pass(db):
    """Per kernel (template head + its full name's template arguments folded in by short()): averages of the
    MFMA-busy pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE) and the
    quantities derived from them (MI355X_MICROARCH.md):
      eff_clock_ghz   = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time (reads high below ~0.3 ms dispatches)
      mfma_busy_frac  = SQ_VALU_MFMA_BUSY_CYCLES (summed over the 1024 SIMDs) / (1024 x GRBM_GUI_ACTIVE / 8),
                        the share of SIMD-cycles of the dispatch in which the MFMA pipe was busy
      mfma_busy_of_peak = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x wall x 2.4 GHz): the same busy cycles against
                        the nominal clock (no GRBM window: the fraction of the dense MFMA peak kept busy)"""
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, count(*), avg(value), avg(duration) from counters_collection "
                     "group by kernel_name, counter_name").fetchall()
    out = {}
    for name, ctr, n, v, dur in rows:
        e = out.setdefault(inst(name), {"launches": int(n), "avg_ns": float(dur)})
        e[ctr] = float(v)
    for k, e in out.items():
        g = e.get("GRBM_GUI_ACTIVE")
        if g:
            cyc = g / 8.0
            e["eff_clock_ghz"] = round(cyc / e["avg_ns"], 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in e:
                e["mfma_busy_frac"] = round(e["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cyc), 4)
                e["mfma_busy_of_peak"] = round(e["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * e["avg_ns"] * 2.4), 4)
            if "SQ_BUSY_CYCLES" in e:
                e["sq_busy_frac"] = round(e["SQ_BUSY_CYCLES"] / (8.0 * cyc), 4)
    return out


def inst(name: str) -> str:
    """short() plus the first template arguments, so the instances of one kernel stay apart."""
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    m = re.match(r"^([\w:]+<[^()]*?>)", n)
    return m.group(1) if m else short(name)


def pmc_pass_check(fe, chk, peak=2516.6):
    """Launch-weighted per-dispatch average of the line's kernel (gemm256_kernel<0, 0, ...> instances) in the
    FETCH_SIZE pass, and the frac each of the three timings implies at the line's FLOP per launch."""
    tot = n = 0
    for k, e in fe.items():
        if k.startswith("gemm256_kernel<0, 0,"):
            tot += e["avg_ns"] * e["launches"]
            n += e["launches"]
    out = {"what": "FETCH_SIZE pass: launch-weighted dispatch average over the gemm256_kernel<0, 0, ...> instances",
           "avg_us": round(tot / n / 1e3, 2) if n else None}
    plain = chk.get("bench_roofline_plain") or {}
    fl = plain.get("flop_per_launch")
    if fl and n:
        ins = chk["in_step"]["avg_us_trace"].get("gemm256_kernel<0,0>")
        out["frac"] = {"line": plain.get("frac"),
                       "trace_in_step": round(fl / (ins * 1e-6) / 1e12 / peak, 4) if ins else None,
                       "pmc_pass": round(fl / (tot / n * 1e-9) / 1e12 / peak, 4)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--command", default="")
    ap.add_argument("--sq", default=None, help="rocpd database of the MFMA-busy pass (SQ_VALU_MFMA_BUSY_CYCLES "
                    "SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE)")
    ap.add_argument("--trace-csv", default=None, help="kernel trace CSV of the same run: the GEMM launches of "
                    "bench.py's roofline replay (after the last AdamW) averaged per (kernel, a_layout, b_layout)")
    ap.add_argument("--bench-json", default=None, help="bench.py output line of the traced run")
    ap.add_argument("--bench-plain", default=None, help="bench.py output line of an un-profiled run of the same command")
    a = ap.parse_args()
    if a.trace_csv:
        import collections
        import csv
        rows = sorted(csv.DictReader(open(a.trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
        last = max(i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"])
        d = collections.defaultdict(list)
        spans = collections.defaultdict(list)
        for r in rows[last + 1:]:
            m = re.search(r"(gemm256_kernel|gemm_bf16_kernel)<(\d), (\d)", r["Kernel_Name"])
            if m:
                k = f"{m.group(1)}<{m.group(2)},{m.group(3)}>"
                d[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                spans[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        # the replay issues every kernel instance's launches back to back (a warm pass, then the timed
        # passes): consecutive dispatches overlap (the next one's waves start while the last tiles of
        # the previous drain), so the per-dispatch average over-counts what the bench's event pair
        # spans; first start -> last end of the timed passes / their launches is the comparable number
        def span_per_launch(v):
            if len(v) < 8 or len(v) % 4:
                return None
            t = v[len(v) // 4:]
            return round((t[-1][1] - t[0][0]) / len(t) / 1e3, 2)
        # the in-step launches the line's achieved / frac come from: the eager probe steps, each behind a
        # torch.cuda._sleep spin (spin_kernel), up to the last AdamW
        first_spin = min((i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]), default=None)
        ins = collections.defaultdict(list)
        if first_spin is not None:
            for r in rows[first_spin:last + 1]:
                m = re.search(r"(gemm256_kernel|gemm_bf16_kernel)<(\d), (\d)", r["Kernel_Name"])
                if m:
                    ins[f"{m.group(1)}<{m.group(2)},{m.group(3)}>"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        chk = {"source": "rocprofv3 --kernel-trace of bench.py",
               "in_step": {"what": "launches of the eager probe steps (first spin_kernel .. last AdamW): the "
                                   "launches the line's roofline.avg_launch_us times with HIP event pairs",
                           "avg_us_trace": {k: round(sum(v) / len(v) / 1e3, 2) for k, v in sorted(ins.items())},
                           "launches_trace": {k: len(v) for k, v in sorted(ins.items())}},
               "replay": {"what": "the roofline replay launches (after the last AdamW): avg_launch_us_isolated_replay",
                          "avg_us_trace": {k: round(sum(v) / len(v) / 1e3, 2) for k, v in sorted(d.items())},
                          "span_per_launch_us_trace": {k: span_per_launch(v) for k, v in sorted(spans.items())},
                          "launches_trace": {k: len(v) for k, v in sorted(d.items())}}}
        if a.bench_json:
            line = [x for x in open(a.bench_json) if x.startswith("{")][-1]
            rf = json.loads(line).get("roofline", {})
            chk["bench_roofline_under_profiler"] = {"kernel": rf.get("kernel"), "avg_launch_us": rf.get("avg_launch_us"),
                                                    "avg_launch_us_isolated_replay": rf.get("avg_launch_us_isolated_replay")}
        if a.bench_plain:
            line = [x for x in open(a.bench_plain) if x.startswith("{")][-1]
            rf = json.loads(line).get("roofline", {})
            chk["bench_roofline_plain"] = {"kernel": rf.get("kernel"), "avg_launch_us": rf.get("avg_launch_us"),
                                           "frac": rf.get("frac"), "flop_per_launch": rf.get("flop_per_launch"),
                                           "avg_launch_us_isolated_replay": rf.get("avg_launch_us_isolated_replay")}
    ks = kernel_stats(a.trace)
    fe, wr = pmc(a.fetch, "FETCH_SIZE"), pmc(a.write, "WRITE_SIZE")
    if a.trace_csv:
        chk["pmc_pass"] = pmc_pass_check(fe, chk)
        with open(a.out + "_roofline_check.json", "w") as f:
            json.dump(chk, f, indent=1)
        print(json.dumps(chk))
    out = {"command": a.command,
           "correction": "hbm_bytes = 2 * FETCH_SIZE + WRITE_SIZE, both KiB (gfx950: FETCH_SIZE counts half of "
                         "16-B/lane streaming reads; MI355X_MICROARCH.md HBM section)",
           "kernels": {}}
    trace_avg = {s: avg for s, _, n, tot, avg, pct in ks}
    for k in sorted(set(fe) | set(wr), key=lambda k: -(fe.get(k, {}).get("avg_kib", 0) * fe.get(k, {}).get("launches", 0))):
        f_, w_ = fe.get(k), wr.get(k)
        e = {"launches": (f_ or w_)["launches"], "avg_us_pmc_pass": round((f_ or w_)["avg_ns"] / 1e3, 3),
             "fetch_kib_per_launch": None if f_ is None else round(f_["avg_kib"], 1),
             "write_kib_per_launch": None if w_ is None else round(w_["avg_kib"], 1),
             "avg_us_trace": None if k not in trace_avg else round(trace_avg[k], 3)}
        if f_ is not None and w_ is not None:
            e["hbm_bytes_per_launch"] = round((2 * f_["avg_kib"] + w_["avg_kib"]) * 1024)
        out["kernels"][k] = e
    if a.sq:
        sq = sq_pass(a.sq)
        out["mfma_pass"] = {
            "counters": "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE (one pass of their own)",
            "derived": "eff_clock_ghz = GRBM_GUI_ACTIVE/8/wall; mfma_busy_frac = MFMA_BUSY/(1024 SIMDs x GRBM_GUI_ACTIVE/8)",
            "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in e.items()}
                        for k, e in sorted(sq.items(), key=lambda kv: -kv[1]["avg_ns"] * kv[1]["launches"])[:40]}}
    with open(a.out + "_pmc.json", "w") as f:
        json.dump(out, f, indent=1)
    for s, _, n, tot, avg, pct in ks[:12]:
        print(f"{s:60s} {n:6d} {avg:9.2f} us {pct:6.2f}%")


if __name__ == "__main__":
    main()
