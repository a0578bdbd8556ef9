#!/usr/bin/env python3
"""Per-kernel ISA statistics from `make asm`'s build/rt_trace.s: instruction count, scratch
(spill) loads/stores, v_readlane/v_writelane (SGPR spills), for the kernels matching a regex.
    python tools/isa_stats.py [regex on the demangled name]"""
import re
import subprocess
import sys

path = "ray-tracer-from-scratch_amd/build/rt_trace.s"
pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else r"kno::k_trace<3, false, true, true, 8>")
s = open(path).read()
for m in re.finditer(r"^(_Z\S+):\s*; @", s, flags=re.M):
    name = m.group(1)
    dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    if not pat.search(dn):
        continue
    j = s.index(".Lfunc_end", m.end())
    body = s[m.end():j]
    ins = [ln.split()[0] for ln in body.splitlines()
           if ln.startswith("\t") and not ln.startswith("\t.") and ln.strip() and not ln.strip().startswith(";")]
    cnt = lambda p: sum(1 for x in ins if x.startswith(p))
    print(f"{dn.replace('rt::', '')[:70]:70s} instr {len(ins):6d} scratch_st {cnt('scratch_store'):3d} "
          f"scratch_ld {cnt('scratch_load'):3d} writelane {cnt('v_writelane'):3d} readlane {cnt('v_readlane'):4d} "
          f"valu {cnt('v_'):5d} salu {cnt('s_'):5d}")
