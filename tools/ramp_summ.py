#!/usr/bin/env python3
"""Summarise tools/ramp_probe.py --chunk output: per run, the first chunks and the means of
the early and late frames.   python tools/ramp_summ.py FILE.jsonl"""
import json
import sys

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    u = d.get("us_per_frame_by_chunk")
    if not u:
        continue
    print(d.get("feedback"), d.get("warm"), d["host_enqueue_us"], u[:8],
          "early(chunks 1-4):", round(sum(u[1:5]) / 4, 2),
          "late(last 20):", round(sum(u[-20:]) / 20, 2))
