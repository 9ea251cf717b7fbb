"""Memory-access audit of the library's gfx950 code object (no GPU needed).

Every pointer a product kernel dereferences reaches it as a buffer resource
(cksum_device.h: `Arr`, `rsrc_of`), so the hardware range-checks every load,
store and atomic against the extent the resource carries: an out-of-range
index reads zeros or is dropped, it can never fault.  This tool reads the
built library's code object and lists, per kernel, every instruction that is
NOT range-checked that way:

  * global_* / flat_* / scratch_* memory instructions (an address in VGPRs or
    SGPRs with no bounds: a stale or wrong index faults);
  * scalar loads whose base is not the kernel-argument segment (s_load from a
    user pointer: no bounds either);
  * scalar-cache writes (s_store / s_atomic / s_dcache_wb / s_buffer_store),
    which no kernel here may contain at all.

    python tools/isa_audit.py [libmicksum.so]       # table of findings
tests/test_isa_audit.py runs the same check on every build.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile
from collections import Counter, OrderedDict

LLVM = "/opt/rocm/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(ROOT, "libunsod_amd", "lib", "libmicksum.so")

UNCHECKED = re.compile(r"^(global|flat|scratch)_\w+")
SCALAR_WRITE = re.compile(r"^s_(store|atomic|buffer_store|buffer_atomic|dcache_wb|scratch_store)\w*")


def code_object(lib: str, out_dir: str) -> str:
    fat = os.path.join(out_dir, "fatbin.bin")
    co = os.path.join(out_dir, "co.elf")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat], check=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


# instructions whose first operand is a source, not a destination
NO_DEST = re.compile(r"^(s_cmp|s_cmpk|s_bitcmp|s_cbranch|s_branch|s_waitcnt|s_setpc|s_nop|s_sleep|s_trap|s_setprio)")
SREG = re.compile(r"^s(\d+)$|^s\[(\d+):(\d+)\]$")


def _sregs(tok: str):
    m = SREG.match(tok)
    if not m:
        return []
    if m.group(1) is not None:
        return [int(m.group(1))]
    return list(range(int(m.group(2)), int(m.group(3)) + 1))


def _transfer(state: frozenset, op: str, ops: list, kernel: str, found: "OrderedDict[str, Counter]", report: bool):
    """One instruction's effect on the set of places (SGPR numbers, VGPR-lane
    pairs) that hold the kernel-argument segment pointer; scalar loads through
    anything else are reported (when `report`)."""
    st = set(state)
    if op.startswith("s_load_dword"):
        base = _sregs(ops[1]) if len(ops) > 1 else []
        if report and (not base or not all(r in st for r in base)):
            found[kernel]["s_load from " + ops[1]] += 1
        st.difference_update(_sregs(ops[0]))
    elif op == "v_writelane_b32" and len(ops) >= 3:
        src = _sregs(ops[1])
        if src and src[0] in st:
            st.add((ops[0], ops[2]))
        else:
            st.discard((ops[0], ops[2]))
    elif op == "v_readlane_b32" and len(ops) >= 3:
        if (ops[1], ops[2]) in st:
            st.update(_sregs(ops[0]))
        else:
            st.difference_update(_sregs(ops[0]))
    elif op == "s_and_b32" and len(ops) == 3 and ops[2] == "0xffff" and _sregs(ops[1]) and _sregs(ops[1])[0] in st:
        # the high half masked to 16 bits (a 48-bit address: the same value),
        # as a buffer resource's base field holds it -- the compiler copies
        # the pointer back out of it
        st.update(_sregs(ops[0]))
    elif op in ("s_mov_b64", "s_mov_b32") and len(ops) >= 2:
        dst, src = _sregs(ops[0]), _sregs(ops[1])
        if src and len(src) == len(dst) and all(r in st for r in src):
            st.update(dst)
        else:
            st.difference_update(dst)
    elif ops and _sregs(ops[0]) and not NO_DEST.match(op):
        st.difference_update(_sregs(ops[0]))
    elif ops and re.match(r"^v\d+$", ops[0]):
        # a VGPR written wholesale loses any lanes it held
        st = {x for x in st if not (isinstance(x, tuple) and x[0] == ops[0])}
    return frozenset(st)


def _kernel_findings(name: str, insns: list, found: "OrderedDict[str, Counter]") -> None:
    """Forward must-dataflow over the kernel's control-flow graph: a place
    holds the kernel-argument pointer at a point iff it does on every path
    there (branch targets from llvm-objdump --symbolize-operands)."""
    # basic blocks: split at labels and after branches
    blocks, labels, cur = [], {}, []
    for kind, a, b in insns:
        if kind == "label":
            if cur:
                blocks.append(cur)
            cur = []
            labels[a] = len(blocks)
            continue
        cur.append((a, b))
        if a.startswith("s_branch") or a.startswith("s_cbranch") or a == "s_endpgm":
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    succ = []
    for i, bl in enumerate(blocks):
        op, ops = bl[-1]
        s = []
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            t = ops[0] if ops else ""
            if t in labels:
                s.append(labels[t])
        if not (op.startswith("s_branch") or op == "s_endpgm") and i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    preds = [[] for _ in blocks]
    for i, ss in enumerate(succ):
        for j in ss:
            preds[j].append(i)
    # entry: the base of the first scalar load is the kernel-argument pointer
    entry = frozenset()
    for bl in blocks:
        for op, ops in bl:
            if op.startswith("s_load_dword"):
                entry = frozenset(_sregs(ops[1]))
                break
        if entry:
            break
    TOP = None
    out = [TOP] * len(blocks)
    work = list(range(len(blocks)))
    while work:
        i = work.pop(0)
        ins = [out[p] for p in preds[i] if out[p] is not TOP] if i else []
        st = entry if i == 0 else (frozenset.intersection(*ins) if ins else TOP)
        if st is TOP:
            continue
        for op, ops in blocks[i]:
            st = _transfer(st, op, ops, name, found, False)
        if st != out[i]:
            out[i] = st
            work.extend(j for j in succ[i] if j not in work)
    for i, bl in enumerate(blocks):
        ins = [out[p] for p in preds[i] if out[p] is not TOP] if i else []
        st = entry if i == 0 else (frozenset.intersection(*ins) if ins else frozenset())
        for op, ops in bl:
            st = _transfer(st, op, ops, name, found, True)


def audit(lib: str = DEFAULT_LIB) -> "OrderedDict[str, Counter]":
    """Kernel -> Counter of its unchecked memory instructions.  The
    kernel-argument segment pointer is followed through SGPR copies and
    spills to VGPR lanes (v_writelane / v_readlane) along the control-flow
    graph; a scalar load through any other SGPRs is reported."""
    with tempfile.TemporaryDirectory() as td:
        co = code_object(lib, td)
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", "--symbolize-operands",
                              co], check=True, capture_output=True, text=True).stdout
    found: "OrderedDict[str, Counter]" = OrderedDict()
    kernels, cur = [], None
    for line in dis.splitlines():
        lab = re.match(r"^[0-9a-f]+ <(L\d+)>:$", line)
        if lab and cur is not None:
            cur[1].append(("label", lab.group(1), None))
            continue
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = (m.group(1), [])
            kernels.append(cur)
            found[cur[0]] = Counter()
            continue
        if cur is None:
            continue
        ins = line.strip().split("//")[0].strip()
        if not ins:
            continue
        op = ins.split()[0]
        ops = [t.strip() for t in ins[len(op):].split(",")] if len(ins) > len(op) else []
        if UNCHECKED.match(op):
            found[cur[0]][op] += 1
        elif SCALAR_WRITE.match(op):
            found[cur[0]]["SCALAR-WRITE " + op] += 1
        cur[1].append(("insn", op, ops))
    for name, insns in kernels:
        _kernel_findings(name, [(k, a, b) if k == "label" else ("insn", a, b) for k, a, b in insns], found)
    return found


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
        return dict(zip(names, out))
    except OSError:
        return {n: n for n in names}


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_LIB
    found = audit(lib)
    bad = {k: v for k, v in found.items() if v}
    names = demangle(list(bad))
    for k, v in bad.items():
        print(f"{names.get(k, k)[:100]:100s} {dict(v)}")
    print(f"{len(found)} kernels, {len(bad)} with unchecked memory instructions")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
