"""Summarize a tools/profile.sh run (gpurun_out/prof_<tag>/) into profiles/.

  python tools/summarize_prof.py <tag>
    -> profiles/rocprof_<tag>_summary.md   kernel stats + PMC-derived numbers
    -> profiles/pmc_traffic.json           per-launch HBM bytes of the steady-state kernels
                                           (read by bench.py for roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE come from
separate --pmc passes, are in KB, and FETCH_SIZE is doubled on gfx950 (it tallies 128-B
requests at 64 B).  Steady-state k_terms launches are the ones with the largest grid
(the pipeline-fill and drain ticks carry fewer regions).
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = name.split("(")[0].replace("bp::", "")
    if name.startswith("void "):
        name = name[5:]
    # k_terms<1>: the pipeline tick (one lane per item); k_terms<2> / <4> / <16>: its drain-tick forms
    # on a lane pair / quad / 16-lane row
    return (name.replace("k_terms<1>", "k_terms").replace("k_terms<2>", "k_terms_pair")
            .replace("k_terms<4>", "k_terms_quad").replace("k_terms<16>", "k_terms_row"))


def load_counters(d):
    path = os.path.join(d, "run_counter_collection.csv")
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(dict)   # dispatch -> {counter: value, kernel, grid}
    for r in rows:
        k = int(r["Dispatch_Id"])
        per[k]["kernel"] = short(r["Kernel_Name"])
        per[k]["grid"] = int(r["Grid_Size"])
        per[k]["vgpr"] = int(r["VGPR_Count"])
        per[k]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return per


def steady(per, kernel):
    ds = [v for v in per.values() if v["kernel"] == kernel]
    if not ds:
        return []
    g = max(v["grid"] for v in ds)
    return [v for v in ds if v["grid"] == g]


def mean(xs):
    return sum(xs) / len(xs) if xs else float("nan")


def prove_summary(tag):
    """tools/profile_prove.sh output -> profiles/rocprof_<tag>_prove_summary.md"""
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_prove")
    stats = list(csv.DictReader(open(os.path.join(base, "trace", "run_kernel_stats.csv"))))
    pmc = {d: load_counters(os.path.join(base, d)) if os.path.isdir(os.path.join(base, d)) else {}
           for d in ("pmc_busy", "pmc_valu", "pmc_fetch", "pmc_write")}
    try:
        bt = json.loads(open(os.path.join(base, "bench_trace.json")).read().strip().splitlines()[-1])
        pv = bt.get("prove") or {}
    except (OSError, ValueError, IndexError):
        pv = {}
    lines = [f"# rocprofv3 summary — prover, {tag}", "",
             "Command: `tools/profile_prove.sh " + tag + "` on one MI355X: bench.py's prove leg (B = "
             f"{pv.get('batch', '?')} 64-bit proofs per hipbp_batch_generate_range_proof batch, K = "
             f"{pv.get('prefix_bits', '?')} prefix tables, {pv.get('streams', '?')} streams, 2 timed + 1 warm-up "
             "batch), after a short verify leg whose kernels are not listed.",
             "", f"Prove leg in the traced run: {pv.get('value', float('nan')):.0f} proofs/s "
             f"({pv.get('ms_per_batch', float('nan')):.1f} ms per batch of {pv.get('batch', '?')}), "
             f"deterministic across streams: {pv.get('deterministic_across_streams')}.", "",
             "## Kernel trace (`rocprofv3 --kernel-trace --stats`) and PMC per launch (mean over launches)", "",
             "| kernel | calls | avg ms | total ms | VALUBusy % | VALU instr/wave | HBM MB/launch (2xFETCH+WRITE) |",
             "|---|---|---|---|---|---|---|"]

    def per(d, k, f):
        return [f(v) for v in pmc[d].values() if v["kernel"] == k]
    for r in stats:
        k = short(r["Name"])
        if not k.startswith("k_prove"):
            continue
        b = per("pmc_busy", k, lambda v: v.get("VALUBusy", float("nan")))
        vi = per("pmc_valu", k, lambda v: v.get("SQ_INSTS_VALU", 0) / v["SQ_WAVES"] if v.get("SQ_WAVES") else float("nan"))
        fe = per("pmc_fetch", k, lambda v: v.get("FETCH_SIZE", float("nan")))
        wr = per("pmc_write", k, lambda v: v.get("WRITE_SIZE", float("nan")))
        hbm = (2 * mean(fe) + mean(wr)) * 1024 / 1e6 if fe and wr else float("nan")
        lines.append(f"| {k} | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{mean(b):.1f} | {mean(vi):.0f} | {hbm:.1f} |")
    lines += ["", "Per batch: prep, sort, terms0 (all A/S terms: the heavy scalar-mults, prefix tables for "
              "the generator bases), chain0, commit, terms1, tx, then per IPA round rterms / chain / round, final. "
              "The commit, rterms and chain launches are latency-bound tails (commit: the A11 sequential "
              "accumulations, one lane per proof; rterms: one scalar-mult chain whatever their size); the streams "
              "put one batch's tails under the other batches' terms0, so their kernel times overlap (the "
              "per-launch averages exceed the per-batch wall time).",
              "HBM bytes apply the gfx950 FETCH_SIZE x2 correction (MI355X_MICROARCH.md)."]
    out_md = os.path.join(ROOT, "profiles", f"rocprof_{tag}_prove_summary.md")
    open(out_md, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


def main():
    if len(sys.argv) > 2 and sys.argv[2] == "prove":
        return prove_summary(sys.argv[1])
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    base = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    out_md = os.path.join(ROOT, "profiles", f"rocprof_{tag}_summary.md")
    stats = list(csv.DictReader(open(os.path.join(base, "trace", "run_kernel_stats.csv"))))
    try:   # the prefix-table width the bench ran with (its line's config)
        kbits = json.loads(open(os.path.join(base, "bench_trace.json")).read().strip().splitlines()[-1])[
            "config"]["prefix_tables"]["bits"]
    except (OSError, ValueError, KeyError, IndexError):
        kbits = "?"
    lines = [f"# rocprofv3 summary — {tag}", "",
             "Command: `tools/profile.sh " + tag + "` on one MI355X "
             "(bench.py --no-cpu --no-ipa --no-prove --no-shard --no-host --no-check --no-h2d --no-repeats --table-legs= "
             f"--msm-log2 $MSM_LOG2 under rocprofv3: the headline configuration — B = 1024, n = 64, K = {kbits} prefix "
             "tables, two pipelines, the default 200 timed steps after 2 warm-up steps — the other legs off).", "",
             "## Kernel trace (`rocprofv3 --kernel-trace --stats`)", "",
             "| kernel | calls | avg ms | min ms | max ms | % time |", "|---|---|---|---|---|---|"]
    for r in stats:
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | "
                     f"{float(r['MinNs'])/1e6:.3f} | {float(r['MaxNs'])/1e6:.3f} | {float(r['Percentage']):.1f} |")
    # steady-state launches from the same kernel trace (largest grid = full pipeline ticks), next to
    # the HIP-event average bench.py measured on the verify stream in the same run
    trace = list(csv.DictReader(open(os.path.join(base, "trace", "run_kernel_trace.csv"))))
    try:
        bt = json.loads(open(os.path.join(base, "bench_trace.json")).read().strip().splitlines()[-1])
        ev_kern, ev_ms = bt["roofline"]["kernel"], bt["roofline"]["avg_launch_ms"]
    except (OSError, ValueError, KeyError, IndexError):
        ev_kern, ev_ms = None, None
    lines += ["", "## Steady-state launches (largest grid) from the kernel trace", "",
              "| kernel | launches | grid | avg ms (rocprofv3) | avg ms (bench.py HIP events, same run) |",
              "|---|---|---|---|---|"]
    trace_ms = {}
    for kern in ("k_terms", "k_terms_pair", "k_terms_quad", "k_msm_points", "k_combine", "k_tree"):
        ds = [r for r in trace if short(r["Kernel_Name"]) == kern]
        if not ds:
            continue
        g = max(int(r["Grid_Size_X"]) for r in ds)
        ss = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ds if int(r["Grid_Size_X"]) == g]
        ev = f"{ev_ms:.3f}" if kern == ev_kern and ev_ms else "—"
        lines.append(f"| {kern} | {len(ss)} | {g} | {mean(ss) / 1e6:.3f} | {ev} |")
        trace_ms[kern] = mean(ss) / 1e6
    os.makedirs(os.path.join(ROOT, "profiles", f"raw_{tag}"), exist_ok=True)
    for src, dst in (("trace/run_kernel_stats.csv", "kernel_stats.csv"), ("bench_trace.json", "bench_trace.json")):
        try:
            open(os.path.join(ROOT, "profiles", f"raw_{tag}", dst), "w").write(open(os.path.join(base, src)).read())
        except OSError:
            pass
    fetch = load_counters(os.path.join(base, "pmc_fetch"))
    write = load_counters(os.path.join(base, "pmc_write"))
    valu = load_counters(os.path.join(base, "pmc_valu"))
    cyc = load_counters(os.path.join(base, "pmc_cyc"))
    lines += ["", "## PMC counters, steady-state launches (largest grid), per launch", "",
              "| kernel | launches | grid | VGPR | FETCH_SIZE KB (raw) | WRITE_SIZE KB | HBM bytes (2xFETCH+WRITE) "
              "| SQ_WAVES | VALU instr/wave | SALU instr/wave | LDS instr/wave | eff. clock GHz | VALU cyc/instr/SIMD |",
              "|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for kern in ("k_terms", "k_terms_pair", "k_terms_quad", "k_msm_points", "k_combine", "k_tree", "k_prep_range",
                 "k_prep_ipa"):
        f, w, v, c = steady(fetch, kern), steady(write, kern), steady(valu, kern), steady(cyc, kern)
        if not f:
            continue
        fk = mean([x.get("FETCH_SIZE", 0) for x in f])
        wk = mean([x.get("WRITE_SIZE", 0) for x in w])
        hbm = (2 * fk + wk) * 1024
        waves = mean([x.get("SQ_WAVES", 0) for x in v])
        vi = mean([x.get("SQ_INSTS_VALU", 0) for x in v])
        si = mean([x.get("SQ_INSTS_SALU", 0) for x in v])
        li = mean([x.get("SQ_INSTS_LDS", 0) for x in v])
        grbm = mean([x.get("GRBM_GUI_ACTIVE", 0) for x in c])
        dur = mean([x["dur_ns"] for x in c])
        clock = grbm / 8 / dur if dur else float("nan")        # GRBM_GUI_ACTIVE summed over 8 XCDs
        cyc_per_instr = (grbm / 8) / (vi / 1024) if vi else float("nan")   # 1024 SIMDs
        traffic[kern] = {"bytes_per_launch": hbm, "fetch_kb": fk, "write_kb": wk, "launches": len(f),
                         "valu_instr_per_wave": vi / waves if waves else None, "valu_instr_per_launch": vi,
                         "eff_clock_ghz": clock, "rocprof_avg_ms": trace_ms.get(kern),
                         "serial_cycles_per_instr_per_simd": cyc_per_instr}
        lines.append(f"| {kern} | {len(f)} | {f[0]['grid']} | {f[0]['vgpr']} | {fk:.0f} | {wk:.0f} | {hbm:.3e} | "
                     f"{waves:.0f} | {vi / waves:.0f} | {si / waves:.0f} | {li / waves:.0f} | {clock:.2f} | "
                     f"{cyc_per_instr:.2f} |")
    busy = load_counters(os.path.join(base, "pmc_busy")) if os.path.isdir(os.path.join(base, "pmc_busy")) else {}
    mix = load_counters(os.path.join(base, "pmc_mix")) if os.path.isdir(os.path.join(base, "pmc_mix")) else {}
    if busy:
        lines += ["", "## VALU roofline (the binding resource), steady-state launches", "",
                  "| kernel | VALUBusy % | VALUUtilization % | INT32 VALU instr/wave | INT64 VALU instr/wave | "
                  "dual-issue quad-cycles/wave |", "|---|---|---|---|---|---|"]
        for kern in ("k_terms", "k_terms_pair", "k_terms_quad", "k_msm_points", "k_combine", "k_tree"):
            b, x, v = steady(busy, kern), steady(mix, kern), steady(valu, kern)
            if not b:
                continue
            vb = mean([d.get("VALUBusy", float("nan")) for d in b])
            vu = mean([d.get("VALUUtilization", float("nan")) for d in b])
            waves = mean([d.get("SQ_WAVES", 0) for d in v]) or float("nan")
            i32 = mean([d.get("SQ_INSTS_VALU_INT32", float("nan")) for d in x]) / waves if x else float("nan")
            i64 = mean([d.get("SQ_INSTS_VALU_INT64", float("nan")) for d in x]) / waves if x else float("nan")
            v2 = mean([d.get("SQ_ACTIVE_INST_VALU2", float("nan")) for d in x]) / waves if x else float("nan")
            traffic.setdefault(kern, {}).update({"valu_busy_pct": vb, "valu_utilization_pct": vu,
                                                  "valu2_cycles_per_wave": v2})
            lines.append(f"| {kern} | {vb:.1f} | {vu:.1f} | {i32:.0f} | {i64:.0f} | {v2:.0f} |")
    lines += ["", "Notes:",
              "- `VALU cyc/instr/SIMD` = kernel cycles (GRBM_GUI_ACTIVE/8) / (SQ_INSTS_VALU / 1024 SIMDs): the "
              "issue interval per SIMD, here with the profiler serialising dispatches; k_terms' own point-op loops "
              "sustain ~4.0 in isolation (profiles/valu_step_roof.json, tools/ubench_step.hip).",
              "- HBM bytes apply the gfx950 FETCH_SIZE x2 correction; the loads here are 16-B-per-lane "
              "(dwordx4) gathers of 128-B points, partly served by L2/MALL, so treat absolute bytes as approximate.",
              "- VALUBusy = 100 * SQ_ACTIVE_INST_VALU / CU_NUM / GRBM_GUI_ACTIVE (rocprofv3 derived metric): the share "
              "of kernel time the CUs' vector ALUs are issuing; VALUUtilization = active lanes per VALU instruction."]
    os.makedirs(os.path.dirname(out_md), exist_ok=True)
    open(out_md, "w").write("\n".join(lines) + "\n")
    # the bench configuration the counters belong to: bench.py uses them only for the same one
    cfg = None
    try:
        bc = json.loads(open(os.path.join(base, "bench_valu.json")).read().strip().splitlines()[-1])["config"]
        cfg = {"batch_per_gpu": bc["batch_per_gpu"], "n": bc["n"],
               "prefix_bits": (bc.get("prefix_tables") or {}).get("bits", 0), "pipelines": bc.get("pipelines")}
    except (OSError, ValueError, KeyError, IndexError):
        pass
    json.dump({"tag": tag, "config": cfg, **traffic}, open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"),
              indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
