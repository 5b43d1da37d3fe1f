"""Static check of hipcc output (never the product): an inline-asm ds_read's
destination VGPRs are written when the read RETURNS, but the compiler takes
them as written at the asm statement.  So until an s_waitcnt lgkmcnt(0)
retires the read, no other instruction may read or write those registers:
a use reads stale data, a write is overwritten later (the stream probe's
first versions reused a pending destination as a DMA address and faulted).
Reports, per kernel, every instruction that touches a pending asm-read
destination before such a wait (branches and labels end the window
conservatively).
usage: hipcc ... --save-temps -c x.hip; python scripts/asm_lds_hazards.py x-hip-amdgcn-amd-amdhsa-gfx950.s"""
import re
import sys


def scan(text):
    out = {}
    for f in re.split(r"\n(?=_Z\w+:)", text)[1:]:
        name = f.split(":")[0]
        pend, bad, in_asm = [], [], False
        for i, raw in enumerate(f.split("\n")):
            l = raw.strip()
            if l.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if l.startswith(";;#ASMEND"):
                in_asm = False
                continue
            l = l.split(";")[0].strip()
            if not l:
                continue
            if (l.startswith("s_waitcnt") and re.search(r"lgkmcnt\(0\)", l)) or l.startswith(".LBB") or \
                    l.startswith("s_cbranch") or l.startswith("s_branch") or l.startswith("s_setpc"):
                pend = []
                continue
            rs = set()
            for a, b, c in re.findall(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", l):
                rs.update([int(c)] if c else range(int(a), int(b) + 1))
            m = re.match(r"ds_read\w*\s+v\[(\d+):(\d+)\]", l) or re.match(r"ds_read\w*\s+v(\d+)()\b", l)
            if m and in_asm:
                d = set(range(int(m.group(1)), int(m.group(2) or m.group(1)) + 1))
                if any(d & p for p in pend):
                    bad.append((i, "overlapping destination: " + l))
                addr = rs - d
                if any(r in p for p in pend for r in addr):
                    bad.append((i, "address in a pending destination: " + l))
                pend.append(d)
                continue
            if any(r in p for p in pend for r in rs):
                bad.append((i, l))
        if bad:
            out[name] = bad
    return out


VMEM_LOAD = re.compile(r"(global_load|buffer_load|global_atomic\w*_rtn|flat_load)\w*")


def scan_vmem(text):
    """The same rule for inline-asm global / buffer loads into VGPRs: the
    destination is pending until an s_waitcnt vmcnt(k) with at least k
    vector-memory loads issued after it (loads return in order; stores are
    not counted, so the check stays conservative).  LDS-DMA loads
    (global_load_lds_*) have no VGPR destination and only count as later
    loads."""
    out = {}
    for f in re.split(r"\n(?=_Z\w+:)", text)[1:]:
        name = f.split(":")[0]
        pend, bad, in_asm = [], [], False  # pend: [dest regs, loads issued after]
        for i, raw in enumerate(f.split("\n")):
            l = raw.strip()
            if l.startswith(";;#ASMSTART"):
                in_asm = True
                continue
            if l.startswith(";;#ASMEND"):
                in_asm = False
                continue
            l = l.split(";")[0].strip()
            if not l:
                continue
            if l.startswith(".LBB") or l.startswith("s_cbranch") or l.startswith("s_branch") or \
                    l.startswith("s_setpc"):
                pend = []
                continue
            if l.startswith("s_waitcnt"):
                m = re.search(r"vmcnt\((\d+)\)", l)
                if m:
                    k = int(m.group(1))
                    pend = [p for p in pend if p[1] < k]
                continue
            rs = set()
            for a, b, c in re.findall(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", l):
                rs.update([int(c)] if c else range(int(a), int(b) + 1))
            is_load = VMEM_LOAD.match(l) is not None
            if is_load:
                for p in pend:
                    p[1] += 1
            lds = "_lds_" in l.split()[0] or " lds" in l
            m = re.match(r"\w+\s+v\[(\d+):(\d+)\]", l) or re.match(r"\w+\s+v(\d+)()\b", l)
            if is_load and in_asm and not lds and m:
                d = set(range(int(m.group(1)), int(m.group(2) or m.group(1)) + 1))
                if any(d & p[0] for p in pend):
                    bad.append((i, "overlapping destination: " + l))
                addr = rs - d
                if any(r in p[0] for p in pend for r in addr):
                    bad.append((i, "address in a pending destination: " + l))
                pend.append([d, 0])
                continue
            if any(r in p[0] for p in pend for r in rs):
                bad.append((i, l))
        if bad:
            out[name] = bad
    return out


if __name__ == "__main__":
    total = 0
    for path in sys.argv[1:]:
        text = open(path).read()
        for name, bad in list(scan(text).items()) + list(scan_vmem(text).items()):
            total += len(bad)
            print(f"{path}: {name[:80]}: {len(bad)}")
            for i, l in bad[:4]:
                print(f"    line {i}: {l}")
    print("hazards:", total)
    sys.exit(1 if total else 0)
