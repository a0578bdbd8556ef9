#!/usr/bin/env python3
"""Turn a tools/make_profiles.sh run (gpurun_out/prof_<round>) into the committed
profiles/<round>/ files and profiles/pmc_traffic.json (bench.py's roofline.traffic).

HBM bytes per launch = FETCH_SIZE * 2 (gfx950 reports half of wide coalesced reads:
MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both KiB * 1024; medians over the 5 dispatches.
"""
import csv
import glob
import json
import os
import re
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    vals = {}
    durs = {}
    for r in csv.DictReader(open(path)):
        if "k_trace" not in r["Kernel_Name"] or "kst::" in r["Kernel_Name"]:  # sampled frames
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        durs[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {k: statistics.median(v) for k, v in vals.items()}
    if durs:
        out["_kernel_ns"] = statistics.median(durs.values())
    return out


N_SIMD = 1024      # MI355X: 256 CUs x 4 SIMDs
N_XCD = 8
F_MAX_GHZ = 2.4    # MI355X_MICROARCH.md: max clock


def valu_hw(c):
    """Measured VALU activity of one dispatch (the verdict's hardware view beside the
    algorithmic roofline_valu): SQ_ACTIVE_INST_VALU counts, per wave, the quad-cycles
    (4 cycles) in which it has a VALU instruction issued; summed over waves and divided by
    the SIMD count it is the VALU-issue cycles per SIMD, priced against the dispatch's
    cycles at the measured clock (GRBM_GUI_ACTIVE is summed over the 8 XCDs).  Lane
    utilisation = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU): the active fraction
    of each issued instruction's 64 lanes (divergence, dead lanes)."""
    need = ("SQ_ACTIVE_INST_VALU", "SQ_THREAD_CYCLES_VALU", "GRBM_GUI_ACTIVE", "SQ_WAVES",
            "SQ_INSTS_VALU", "SQ_INSTS_SALU", "_kernel_ns")
    if not all(k in c for k in need):
        return None
    ns = c["_kernel_ns"]
    ghz = c["GRBM_GUI_ACTIVE"] / N_XCD / ns
    # priced at the maximum clock: a lower bound on the busy fraction when the clock ran lower
    busy = c["SQ_ACTIVE_INST_VALU"] * 4 / N_SIMD / (ns * F_MAX_GHZ)
    lanes = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])
    w = c["SQ_WAVES"]
    return {"valu_busy": round(busy, 3), "valu_lane_util": round(lanes, 3),
            "valu_busy_x_lanes": round(busy * lanes, 3),
            "valu_insts_per_wave": round(c["SQ_INSTS_VALU"] / w, 1),
            "salu_insts_per_wave": round(c["SQ_INSTS_SALU"] / w, 1),
            "smem_insts_per_wave": round(c.get("SQ_INSTS_SMEM", 0) / w, 1),
            "branch_insts_per_wave": round(c.get("SQ_INSTS_BRANCH", 0) / w, 1),
            "clock_ghz_grbm": round(ghz, 3), "kernel_ns_profiled": ns,
            "formula": "busy = SQ_ACTIVE_INST_VALU*4/1024/(kernel_ns*2.4 GHz) (max clock: a lower "
                       "bound); lanes = SQ_THREAD_CYCLES_VALU/(64*SQ_ACTIVE_INST_VALU); medians "
                       "of 5 dispatches under rocprofv3 --pmc"}


def main(rnd="r01"):
    src = os.path.join(REPO, "gpurun_out", f"prof_{rnd}")
    dst = os.path.join(REPO, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "bench", "**", "*.csv"), recursive=True):
        if re.search(r"(kernel_stats|kernel_trace|agent_info)", f):
            shutil.copy(f, os.path.join(dst, "bench_" + os.path.basename(f)))
    bj = os.path.join(src, "bench.json")
    if os.path.exists(bj):
        shutil.copy(bj, os.path.join(dst, "bench_under_rocprof.json"))
    for run in ("bench_fif1", "bench_default"):  # one-stream bench, the driver's command
        for f in glob.glob(os.path.join(src, run, "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(dst, f"{run}_kernel_stats.csv"))
        if os.path.exists(os.path.join(src, run + ".json")):
            shutil.copy(os.path.join(src, run + ".json"), os.path.join(dst, f"{run}_under_rocprof.json"))
    sys.path.insert(0, os.path.join(REPO, "ray-tracer-from-scratch_amd"))
    from rtamd import scenes
    traffic_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    traffic = json.load(open(traffic_path)) if os.path.exists(traffic_path) else {}
    valu_path = os.path.join(REPO, "profiles", "pmc_valu.json")
    valu = json.load(open(valu_path)) if os.path.exists(valu_path) else {}
    summary = {}
    for d in sorted(glob.glob(os.path.join(src, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        _, cfg, prec, tag = os.path.basename(d).split("_", 3)
        files = glob.glob(os.path.join(d, "**", "pmc_counter_collection.csv"), recursive=True)
        if not files:
            continue
        c = counters(files[0])
        summary.setdefault(cfg, {}).setdefault(prec, {}).update(c)
        shutil.copy(files[0], os.path.join(dst, f"pmc_{cfg}_{prec}_{tag}.csv"))
    for cfg, per in summary.items():
        cf = scenes.CONFIGS[cfg]
        sc = cf.scene()
        n_sph = sum(1 for o in sc if o.kind == 0)
        workload = f"{cfg}:{cf.width}x{cf.height}:d{cf.depth}:s{n_sph}w{len(sc) - n_sph}"
        for prec, c in per.items():
            hw = valu_hw(c)
            if hw is not None:
                hw["source"] = f"profiles/{rnd}/pmc_{cfg}_{prec}_*.csv"
                valu.setdefault(workload, {})[prec] = hw
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
                traffic.setdefault(workload, {})[prec] = {
                    "hbm_bytes_per_launch": hbm,
                    "fetch_size_kib": c["FETCH_SIZE"], "write_size_kib": c["WRITE_SIZE"],
                    "source": f"profiles/{rnd}/pmc_{cfg}_{prec}_*.csv",
                }
    json.dump(traffic, open(traffic_path, "w"), indent=1, sort_keys=True)
    json.dump(valu, open(valu_path, "w"), indent=1, sort_keys=True)
    print(json.dumps(valu, indent=1))
    json.dump(summary, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
