"""Measurement/audit tool (not product): scan hipcc's gfx950 assembly for a
VMEM store of more than 8 bytes (dwordx3 / dwordx4, global / buffer / flat)
whose data VGPRs are rewritten by the very next instruction -- the
store-data hazard behind round 1's buffer-store corruption (the 4th dword of
a buffer_store_dwordx4 with an SGPR soffset rewritten by the next VALU op).
usage: store_hazard_check.py file.s [...]  -> one line per hit, exit 1 if any"""
import re
import sys

STORE = re.compile(r"^\s*(global|buffer|flat)_store_dwordx([34])\s+(?:v\[\d+:\d+\],\s*)?v\[(\d+):(\d+)\]")
BSTORE = re.compile(r"^\s*buffer_store_dwordx([34])\s+v\[(\d+):(\d+)\]")
DST = re.compile(r"^\s*(v_\S+|ds_read\S*|global_load\S*|buffer_load\S*|flat_load\S*)\s+v(?:\[(\d+):(\d+)\]|(\d+))")


def data_regs(line):
    m = BSTORE.match(line)
    if m:
        return int(m.group(2)), int(m.group(3))
    m = re.match(r"^\s*(global|flat)_store_dwordx([34])\s+v(?:\[\d+:\d+\]|\d+),\s*v\[(\d+):(\d+)\]", line)
    if m:
        return int(m.group(3)), int(m.group(4))
    return None


def main(paths):
    hits = 0
    for p in paths:
        fn = None
        lines = [l for l in open(p).read().split("\n")]
        body = []
        for l in lines:
            m = re.match(r"^(\S+):\s*(;.*)?$", l)
            if m and not l.startswith("."):
                fn = m.group(1)
            s = l.strip()
            if not s or s.startswith(";") or s.startswith("."):
                continue
            body.append((fn, s))
        for k, (fn, s) in enumerate(body[:-1]):
            r = data_regs(s)
            if not r:
                continue
            nxt = body[k + 1][1]
            m = DST.match(nxt)
            if not m:
                continue
            a, b = (int(m.group(4)), int(m.group(4))) if m.group(4) else (int(m.group(2)), int(m.group(3)))
            if not (b < r[0] or a > r[1]):
                hits += 1
                print(f"{p}: {fn}: '{s}' then '{nxt}'")
    print(f"{hits} hazard(s)")
    return 1 if hits else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
