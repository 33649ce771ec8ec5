#!/usr/bin/env python3
"""Per-kernel ISA statistics of kernels.hip (device-only asm): cross-lane op counts,
vmcnt(0) waits, VGPRs, occupancy.  Usage: isa_stats.py k.s [name-filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else "k_matvec"
for m in re.finditer(r"\n(_ZN4llmi\w+):[^\n]*\n(.*?)\.Lfunc_end", s, re.S):
    name, body = m.groups()
    if flt not in name:
        continue
    tail = s[m.end():m.end() + 4000]
    vg = re.search(r"; NumVgprs: (\d+)", tail)
    occ = re.search(r"; Occupancy: (\d+)", tail)
    sp = re.search(r"; ScratchSize: (\d+)", tail)
    print(f"{name[:48]:48s} bperm {body.count('ds_bpermute'):3d} dpp {body.count('_dpp'):3d} "
          f"permlane {body.count('permlane'):3d} vmcnt0 {body.count('vmcnt(0)'):3d} instr {body.count(chr(10)):5d} "
          f"vgpr {vg.group(1) if vg else '?'} occ {occ.group(1) if occ else '?'} scratch {sp.group(1) if sp else '?'}")
