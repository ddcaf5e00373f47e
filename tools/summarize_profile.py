#!/usr/bin/env python3
"""Summarise a tools/gpu.sh profile run into profiles/ (committed evidence).

Writes profiles/<tag>_<config>_<schedule>_f<prec>.md (kernel stats table + PMC
traffic) and profiles/pmc_<config>_<schedule>_f<prec>.json (HBM bytes per batch
of each phase bench.py times -- "score", "fold_phase", "apply", "relowner" --
and per launch of each kernel family; read by bench.py for roofline.traffic).
The PMC passes run `batches` batches (warmup + steps of the pass).

HBM bytes per MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts exactly half of a wide coalesced read, so the
corrected read bytes are 2 * FETCH_SIZE * 1024 (uncalibrated for other access
widths -- both raw and corrected values are recorded).
"""
import csv
import json
import os
import sys
from collections import defaultdict

FAMILY = {"transe_fold_long_kernel": "fold_long", "transe_fold_kernel": "fold", "transe_score_kernel": "score",
          "relowner": "relowner", "transh_owner": "relowner", "transr_owner": "relowner",
          "transh_score": "score", "transr_project": "score", "transr_compat": "score", "ticket": "tickets",
          "relowner_desc": "desc", "relowner_compact": "desc", "transr_commit": "commit"}


# kernel -> the bench.py phase it belongs to (the HIP-event spans of the engine)
PHASE = [("transe_score", "score"), ("transh_score", "score"), ("transr_project", "score"),
         ("transr_compat", "score"), ("transr_tile", "score"), ("rpar_scan", "score"),
         ("transr_proj_wave", "score"), ("transr_grad_wave", "score"), ("transr_rows", "apply"),
         ("transr_cons", "apply"),
         ("transe_fold", "fold_phase"), ("transe_apply", "fold_phase|apply"), ("transh_w_apply", "fold_phase"),
         ("transh_orth", "fold_phase"), ("transr_rel_rows", "apply"), ("transr_entity", "apply"),
         ("transr_constraint", "apply"), ("owner_kernel", "relowner"), ("owner_reg_kernel", "relowner")]


def family(name):
    for k, v in FAMILY.items():
        if k in name:
            return v
    return name


def phase(name):
    for k, v in PHASE:
        if k in name:
            return v
    return None


CLOCK_HZ, SIMDS, XCDS = 2.4e9, 1024, 8  # MI355X_MICROARCH.md: 256 CUs x 4 SIMDs in 8 XCDs
PEAK_F64_MFMA_TFLOPS = 78.6  # v_mfma_f64_16x16x4_f64: 64 cycles / 2048 FLOP per SIMD, 1024 SIMDs, 2.4 GHz


def mfma_table(src, stats):
    """f64 MFMA work and utilisation per kernel from the SQ_INSTS_VALU_MFMA_MOPS_F64
    / SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass (rocprofv3 derived-counter
    formulas: MfmaFlopsF64 = MOPS_F64 x 512).  SQ_VALU_MFMA_BUSY_CYCLES is summed over
    all 1024 SIMDs and GRBM_GUI_ACTIVE over the 8 XCDs, so the utilisation is
    BUSY / (kernel cycles x 1024 SIMDs) with kernel cycles = the rocprofv3 average
    duration x 2.4 GHz (mfma_util_pct) or GUI_ACTIVE / 8 (mfma_util_pct_gui)."""
    path = os.path.join(src, "pmc_MFMA", "run_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k][r["Counter_Name"]] += 1
    avg_us = {r["Name"].split("(")[0].split("<")[0].strip(): float(r["AverageNs"]) / 1e3 for r in stats}
    out = {}
    for k, v in agg.items():
        n = max(cnt[k].values())
        mops = v.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) / n
        if mops <= 0:
            continue
        flops = mops * 512
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / n
        gui = v.get("GRBM_GUI_ACTIVE", 0.0) / n
        us = avg_us.get(k)
        out[k] = {"mfma_f64_flop_per_launch": flops, "avg_us": us,
                  "achieved_tflops": flops / (us * 1e-6) / 1e12 if us else None,
                  "frac_of_f64_mfma_peak": (flops / (us * 1e-6) / 1e12) / PEAK_F64_MFMA_TFLOPS if us else None,
                  "mfma_busy_cycles": busy, "gui_active_cycles": gui,
                  "mfma_util_pct": 100.0 * busy / (us * 1e-6 * CLOCK_HZ * SIMDS) if us else None,
                  "mfma_util_pct_gui": 100.0 * busy / (gui / XCDS * SIMDS) if gui else None}
    return out


def main(src, tag, config, prec, schedule="parallel", batches="200"):
    nbatch = float(batches)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    bench = open(os.path.join(src, "bench.json")).read().strip()
    # PARALLEL TransR sub-batches: a phase-A / phase-B launch pair per sub-batch, so a
    # phase's bytes per launch are its bytes per batch over the sub-batch count
    sub = int(json.loads(bench).get("config", {}).get("sub_batches", 1) or 1)
    nbatch *= sub
    pmc = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        path = os.path.join(src, f"pmc_{c}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        agg = defaultdict(lambda: [0.0, 0])
        ph = defaultdict(float)
        for r in csv.DictReader(open(path)):
            a = agg[family(r["Kernel_Name"])]
            a[0] += float(r["Counter_Value"])
            a[1] += 1
            p = phase(r["Kernel_Name"])
            if config.startswith("transr") and ("transe_" in r["Kernel_Name"] or "long_segments" in r["Kernel_Name"]):
                p = None  # the TransE-init seed run of bench.py, not the measured TransR batches
            for q in (p.split("|") if p else []):
                ph[q] += float(r["Counter_Value"])
        pmc[c] = {k: v[0] / max(1, v[1]) for k, v in agg.items()}  # KiB per launch
        pmc[c + "_phase"] = {k: v / nbatch for k, v in ph.items()}  # KiB per launch (batch or sub-batch)
    per_kernel = {}
    for fam in set(pmc.get("FETCH_SIZE", {})) | set(pmc.get("WRITE_SIZE", {})):
        f = pmc.get("FETCH_SIZE", {}).get(fam, 0.0) * 1024
        w = pmc.get("WRITE_SIZE", {}).get(fam, 0.0) * 1024
        per_kernel[fam] = {"fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes_per_launch": 2 * f + w}
    for p in set(pmc.get("FETCH_SIZE_phase", {})) | set(pmc.get("WRITE_SIZE_phase", {})):
        f = pmc.get("FETCH_SIZE_phase", {}).get(p, 0.0) * 1024
        w = pmc.get("WRITE_SIZE_phase", {}).get(p, 0.0) * 1024
        per_kernel[p] = {"fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes_per_launch": 2 * f + w,
                         "note": f"phase total per launch ({sub} a batch)"}
    mf = mfma_table(src, stats)
    if mf:
        per_kernel["mfma_f64"] = mf
    out_json = os.path.join(root, "profiles", f"pmc_{config}_{schedule}_f{prec}.json")
    json.dump(per_kernel, open(out_json, "w"), indent=1, sort_keys=True)
    lines = [f"# Profile {tag}: {config}, {schedule} schedule (f{prec})", "", "Command: `tools/gpu.sh profile` on one MI355X "
             "(rocprofv3 --kernel-trace --stats; separate --pmc FETCH_SIZE / WRITE_SIZE passes).", "",
             "## bench.py line", "", "```", bench, "```", "", "## Kernel stats (rocprofv3 --stats)", "",
             "| kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|"]
    if config.startswith("transr"):  # not the TransE-init seed run of bench.py
        stats = [r for r in stats if not any(x in r["Name"] for x in ("transe_", "long_segments"))]
    for r in stats[:16]:
        lines.append(f"| {r['Name'][:60]} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    lines += ["", "## HBM traffic per launch (PMC, gfx950-corrected: 2 x FETCH_SIZE + WRITE_SIZE)", "",
              "| kernel family | FETCH_SIZE raw (bytes) | WRITE_SIZE (bytes) | corrected HBM bytes |", "|---|---|---|---|"]
    for fam, v in sorted(((k, v) for k, v in per_kernel.items() if k != "mfma_f64"),
                         key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
        lines.append(f"| {fam} | {v['fetch_bytes_raw']:.0f} | {v['write_bytes']:.0f} | {v['hbm_bytes_per_launch']:.0f} |")
    if mf:
        lines += ["", f"## f64 MFMA per launch (PMC: SQ_INSTS_VALU_MFMA_MOPS_F64 x 512; peak {PEAK_F64_MFMA_TFLOPS} TF)", "",
                  "| kernel | MFMA FLOP | avg us | TFLOP/s | frac of f64 MFMA peak | MfmaUtil % (duration) | MfmaUtil % (GUI_ACTIVE/8) |",
                  "|---|---|---|---|---|---|---|"]
        for k, v in sorted(mf.items(), key=lambda kv: -kv[1]["mfma_f64_flop_per_launch"]):
            lines.append(f"| {k[:50]} | {v['mfma_f64_flop_per_launch']:.3g} | {v['avg_us'] or 0:.1f} | "
                         f"{v['achieved_tflops'] or 0:.2f} | {v['frac_of_f64_mfma_peak'] or 0:.4f} | "
                         f"{v['mfma_util_pct'] or 0:.2f} | {v['mfma_util_pct_gui'] or 0:.2f} |")
    md = os.path.join(root, "profiles", f"{tag}_{config}_{schedule}_f{prec}.md")
    open(md, "w").write("\n".join(lines) + "\n")
    print(md, out_json)


if __name__ == "__main__":
    main(*sys.argv[1:7])
