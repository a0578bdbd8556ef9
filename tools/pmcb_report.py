#!/usr/bin/env python3
"""Report of a tools/pmcb_session.sh run: per setup, kernel time (min of launches 2..5) and
per-wave instruction counts.   python tools/pmcb_report.py gpurun_out/<TAG>"""
import collections
import csv
import json
import sys


def main(d):
    order = json.load(open(f"{d}/order.json"))
    rows = [r for r in csv.DictReader(open(f"{d}/p1/p1_counter_collection.csv"))
            if "k_trace" in r["Kernel_Name"]]
    by = collections.OrderedDict()
    for r in rows:
        by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    disp = list(by.values())
    kt = [r for r in csv.DictReader(open(f"{d}/kt/kt_kernel_trace.csv")) if "k_trace" in r["Kernel_Name"]]
    i = j = 0
    for o in order:
        c = disp[i + o["launches"] - 1]
        i += o["launches"]
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt[j:j + 5]]
        j += 5
        us = min(durs[1:]) / 1e3
        px64 = o["pixels"] / 64.0
        print(f"{o['setup']:16s} us {us:7.1f}  per 64 px: VALU {c['SQ_INSTS_VALU'] / px64:7.1f} "
              f"SALU {c['SQ_INSTS_SALU'] / px64:6.1f} SMEM {c['SQ_INSTS_SMEM'] / px64:5.1f}  "
              f"waves {c['SQ_WAVES']:.0f} wait {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.2f} "
              f"wavecyc/64px {c['SQ_WAVE_CYCLES'] / px64:.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
