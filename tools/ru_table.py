#!/usr/bin/env python3
"""Condense `make asm`'s build/resource_usage.txt to one line per kernel:
name VGPRs SGPRs scratch occupancy.   python tools/ru_table.py [file]"""
import re
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "ray-tracer-from-scratch_amd/build/resource_usage.txt"
cur = None
rows = {}
for line in open(path):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"(TotalSGPRs|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    m = re.match(r"_ZN2rt7k_traceILi(\d)ELb(\d)ELb(\d)ELb(\d)ELi(\d+)E", k)
    name = (f"trace prec={m.group(1)} sun={m.group(2)} int={m.group(3)} cull={m.group(4)} "
            f"maxd={m.group(5)}" if m else k)
    print(f"{name:50s} v{v.get('VGPRs')} s{v.get('TotalSGPRs')} scr{v.get('ScratchSize')} occ{v.get('Occupancy')}")
