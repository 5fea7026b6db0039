"""Scan the built device code for two gfx9 hazards the compiler pads for its own instructions but not around an
inline-asm block (round 5's loader-wave AdamW experiment, DESIGN.md §4, hit both):
  - a VALU write of an SGPR followed within 5 wait states by a vector-memory instruction reading it (a descriptor
    restored from a spill by v_readlane right before an asm buffer store: stale descriptor words, a GPU fault);
  - a vector-memory store of more than 8 bytes followed, with no wait state between, by a VALU write of one of its
    data VGPRs (the store may send the new value: silently corrupted data);
  - an SALU write of M0 directly followed by an LDS-DMA (`... lds`) that takes its LDS address from M0 (one wait
    state needed: the hip guide's LDS-DMA recipe pads it; the DMA statements had not until round 5).
Plus, with --loads, an audit of every vector-memory load into VGPRs: along the fall-through path (up to the next
branch) no instruction may read or write its destination before an s_waitcnt whose vmcnt proves the load complete
(in-order completion: vmcnt(N) with fewer than N+1 operations issued after it).  hipcc's own loads pass by
construction; an inline-asm load (which hipcc does not count) fails it when the compiler copies or reuses the
destination before the kernel's own wait — garbage values, or a fault where the register held an address.

usage: python tools/asm_hazards.py [objects...]   (default: asr-transformer_amd/asrx/lib/*.o; exit 1 on a hit)
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
_REG = re.compile(r"s\[(\d+):(\d+)\]|\bs(\d+)\b")


def _sregs(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(1):
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def _sgpr_defs(inst):
    """SGPRs a VALU instruction writes (lane reads, VOP3 compares, carry / scale outputs)."""
    op, _, args = inst.partition(" ")
    ops = [a.strip() for a in args.split(",")]
    if op.startswith(("v_readlane", "v_readfirstlane")) or (op.startswith("v_cmp") and op.endswith("_e64")):
        return _sregs(ops[0])
    if ("_co_" in op or op.startswith("v_div_scale")) and op.endswith("_e64") and len(ops) > 1:
        return _sregs(ops[1])
    return set()


_VREG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")


def _vregs(text):
    out = set()
    for m in _VREG.finditer(text):
        if m.group(1):
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def scan_text(dis):
    """(line, vmem instruction, writer) for every hit in llvm-objdump / -S output."""
    insts = []
    for ln, raw in enumerate(dis.split("\n"), 1):
        t = raw.split("//")[0].split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":") or t.startswith("<"):
            continue
        insts.append((ln, t))
    hits = []
    for k, (ln, t) in enumerate(insts):
        if not t.startswith(("buffer_", "global_", "tbuffer_")):
            continue
        op = t.split()[0]
        if t.rstrip().endswith(" lds") and k > 0:
            prev = insts[k - 1][1]
            if prev.startswith("s_") and not prev.startswith("s_nop") and prev.partition(" ")[2].split(",")[0].strip() == "m0":
                hits.append((ln, t, prev))
        if "store" in op and op.endswith(("x3", "x4")) and k + 1 < len(insts):
            nxt = insts[k + 1][1]
            data = _vregs(t.partition(" ")[2].split(",")[0] if not op.startswith("global_")
                          else t.partition(" ")[2].split(",")[1])
            if nxt.startswith("v_") and _vregs(nxt.partition(" ")[2].split(",")[0]) & data:
                hits.append((ln, t, nxt))
        reads = _sregs(t.partition(" ")[2])
        ws, j = 0, k - 1
        while j >= 0 and ws < 5:
            lt = insts[j][1]
            if lt.startswith("s_nop"):
                ws += int(lt.split()[1], 0) + 1
            else:
                if lt.startswith("v_") and _sgpr_defs(lt) & reads:
                    hits.append((ln, t, lt))
                ws += 1
            j -= 1
    return hits


_VMEM = ("buffer_", "global_", "tbuffer_", "flat_", "scratch_")
_VMCNT = re.compile(r"vmcnt\((\d+)\)")


def scan_loads(dis, horizon=4000):
    """(line, load, first toucher) for every VGPR load used before a wait that proves it complete."""
    insts = []
    for ln, raw in enumerate(dis.split("\n"), 1):
        t = raw.split("//")[0].split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":") or t.startswith("<"):
            continue
        insts.append((ln, t))
    hits = []
    for k, (ln, t) in enumerate(insts):
        op, _, args = t.partition(" ")
        if not op.startswith(_VMEM) or "load" not in op or t.rstrip().endswith(" lds"):
            continue
        dst = _vregs(args.split(",")[0])
        if not dst:
            continue
        after = 0
        for j in range(k + 1, min(len(insts), k + 1 + horizon)):
            lt = insts[j][1]
            lop, _, largs = lt.partition(" ")
            if lop == "s_waitcnt":
                m = _VMCNT.search(largs)
                if m and int(m.group(1)) < after + 1 and int(m.group(1)) <= after - 0:
                    break
                if m and int(m.group(1)) == 0:
                    break
                continue
            if lop.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                break
            if lop.startswith(_VMEM):
                # a younger LOAD that only overwrites the register (its destination, not its address) is no hazard:
                # loads return in issue order, so the younger value lands last (compiler spill reloads do this)
                lparts = largs.split(",")
                only_dst = "load" in lop and not (_vregs(",".join(lparts[1:])) & dst)
                if _vregs(largs) & dst and not only_dst:
                    hits.append((ln, t, lt))
                    break
                after += 1
                continue
            if _vregs(largs) & dst:
                hits.append((ln, t, lt))
                break
    return hits


def disassemble(obj):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        f"--targets={TARGET}", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                              capture_output=True, text=True).stdout


def main(argv):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    loads = "--loads" in argv
    argv = [a for a in argv if a != "--loads"]
    objs = argv or sorted(glob.glob(os.path.join(root, "asr-transformer_amd", "asrx", "lib", "*.o")))
    bad = 0
    for o in objs:
        dis = disassemble(o)
        hits = scan_text(dis) + (scan_loads(dis) if loads else [])
        for ln, t, w in hits:
            print(f"{os.path.basename(o)}:{ln}: {t}  <-  {w}")
        bad += len(hits)
    print(f"{len(objs)} objects, {bad} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
