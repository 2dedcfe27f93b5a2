#!/usr/bin/env python3
"""Static instruction mix of one kernel in a gfx950 assembly file (hipcc --offload-device-only -S), per basic block,
with the blocks of each loop (a backward branch) summed, and an issue-cycle estimate per class.

usage: isa_mix.py file.s kernel_substring [--blocks]

Issue costs (cycles per wave64 instruction on one SIMD; tools/valu_rates.hip measurements): plain f32 VALU
~2, packed f32 / f64 ~4, transcendental (v_exp/v_rcp/v_sqrt/v_log/v_rsq f32) ~8, f64 transcendental ~16.
"""
import re
import sys

TRANS = re.compile(r"^v_(exp|rcp|sqrt|log|rsq|sin|cos)_(f32|f16)")
TRANS64 = re.compile(r"^v_(rcp|sqrt|rsq)_f64")
F64 = re.compile(r"^v_(fma|mul|add|max|min|ldexp|fract|div_scale|div_fmas|div_fixup|trig_preop)_f64|^v_cvt_f(32|64)_f(64|32)|^v_cmp_\w+_f64|^v_cmpx_\w+_f64|^v_frexp\w*_f64")
PK = re.compile(r"^v_pk_")
DS = re.compile(r"^ds_")
VMEM = re.compile(r"^(buffer|global|flat|scratch)_")
SALU = re.compile(r"^s_")
MFMA = re.compile(r"^v_mfma|^v_smfmac")


def classify(op):
    if MFMA.match(op):
        return "mfma"
    if TRANS64.match(op):
        return "trans64"
    if TRANS.match(op):
        return "trans"
    if F64.match(op) or (op.startswith("v_") and "_f64" in op):
        return "f64"
    if PK.match(op):
        return "pk"
    if op.startswith("v_"):
        return "valu"
    if DS.match(op):
        return "lds"
    if VMEM.match(op):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if SALU.match(op):
        return "salu"
    return "other"


COST = {"valu": 2, "pk": 4, "f64": 4, "trans": 8, "trans64": 16, "mfma": 0}


def kernel_lines(path, name):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(name), l) or
                 (l.startswith("_Z") and name in l.split(":")[0] and l.split(":")[0].endswith(name.split()[-1])))
    end = start
    while not lines[end].strip().startswith("s_endpgm"):
        end += 1
    return lines[start:end + 1]


def blocks(body):
    bl, cur, label = [], [], "entry"
    for l in body[1:]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            bl.append((label, cur))
            label, cur = m.group(1), []
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur.append(t.split(";")[0].strip())
    bl.append((label, cur))
    return bl


def mix(instrs):
    c = {}
    for ins in instrs:
        op = ins.split()[0]
        k = classify(op)
        c[k] = c.get(k, 0) + 1
    return c


def cycles(c):
    return sum(COST.get(k, 0) * v for k, v in c.items())


def main():
    path, name = sys.argv[1], sys.argv[2]
    body = kernel_lines(path, name)
    bl = blocks(body)
    idx = {lab: i for i, (lab, _) in enumerate(bl)}
    loops = []
    for i, (lab, ins) in enumerate(bl):
        for t in ins:
            m = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\S+)", t)
            if m and idx.get(m.group(2), i + 1) <= i:
                loops.append((idx[m.group(2)], i))
    tot = mix([t for _, ins in bl for t in ins])
    print("kernel: %s\ntotal static: %s  (est. issue cycles %d)" % (body[0].split(":")[0][:90], tot, cycles(tot)))
    for a, b in loops:
        c = mix([t for _, ins in bl[a:b + 1] for t in ins])
        print("loop %s..%s (%d blocks): %s  est. cycles %d" % (bl[a][0], bl[b][0], b - a + 1, c, cycles(c)))
    if "--blocks" in sys.argv:
        for lab, ins in bl:
            c = mix(ins)
            print("  %-16s n=%4d %s" % (lab, len(ins), c))


if __name__ == "__main__":
    main()
