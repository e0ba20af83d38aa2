"""k_service's common frame path and its scratch traffic, from the ISA.

Builds pong_ga.hip's device object with line tables (the product's flags plus
-gline-tables-only), disassembles the bench instance
k_service<8,16,3,double,untraced,no-horizon> and reports
  * the common frame path: the straight-line code from the top block's
    "no start, no hidden ball" branch target to the loop's back edge (every
    rare block of the frame is out of line, behind a wave-uniform branch),
    counted by instruction class and by source file -- the path a wave-frame
    takes when every game's ball is in play, no face is reached and every
    certificate passes;
  * every scratch (spill) instruction of the kernel by source line: where the
    register allocator spilled, so that none sits on the common path.

    python tools/isa_frame.py [-DNAME ...] [--dump listing.txt] [> profiles/r05/isa_frame.txt]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "neuro-genetic-pong-self-play_amd", "csrc")
SYM = "_ZN2pg9k_serviceILi8ELi16ELi3EdLb1ELb0EEEvNS_10EvalParamsE"
HIPCC = "/opt/rocm/bin/hipcc"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def disassemble(tmp, defs=()):
    obj = os.path.join(tmp, "k.o")
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                           "-fno-slp-vectorize", "-I", os.path.join(REPO, "include"), "-mllvm",
                           "-amdgpu-sched-strategy=iterative-ilp", "-gline-tables-only", "--cuda-device-only",
                           "--no-gpu-bundle-output", *defs, "-c", "-o", obj, os.path.join(CSRC, "pong_ga.hip")])
    out = subprocess.check_output([OBJDUMP, "-d", "-l", "--no-show-raw-insn", "--disassemble-symbols=" + SYM, obj],
                                  text=True)
    rows, cur = [], "?"
    for ln in out.splitlines():
        m = re.match(r"; (\S+):(\d+)", ln)
        if m:
            cur = os.path.basename(m.group(1)) + ":" + m.group(2)
            continue
        if ln.startswith("\t"):
            ins, _, addr = ln.strip().partition("//")
            a = addr.strip().split(":")[0]
            if a:
                rows.append((int(a, 16), cur, ins.strip()))
    return rows


def branch_target(addr, ins):
    m = re.match(r"s_(?:cbranch_\w+|branch) (\d+)$", ins)
    if not m:
        return None
    off = int(m.group(1))
    off = off - 65536 if off >= 32768 else off
    return addr + 4 + 4 * off


def cls(ins):
    op = ins.split()[0]
    if op.startswith(("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq", "v_sin", "v_cos")):
        return "valu (transcendental)"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("ds_",)):
        return "lds"
    return "memory"


def main():
    # options: -DNAME... (an experiment build's defines), --dump FILE (the annotated listing)
    defs = [a for a in sys.argv[1:] if a.startswith("-D")]
    for i, a in enumerate(sys.argv):  # -mllvm OPTION pairs pass through
        if a == "-mllvm" and i + 1 < len(sys.argv):
            defs += [a, sys.argv[i + 1]]
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    with tempfile.TemporaryDirectory() as tmp:
        rows = disassemble(tmp, defs)
    if dump:
        with open(dump, "w") as fh:
            for a, src, ins in rows:
                fh.write(f"{a:8x}  {src:28s} {ins}\n")
    by_addr = {a: i for i, (a, _, _) in enumerate(rows)}
    # the loop: the last backward conditional branch taken from the `if (top)`
    # test's source line; its fall-through s_branch leads to the common path
    head = None
    for i, (a, src, ins) in enumerate(rows):
        t = branch_target(a, ins)
        if t is not None and ins.startswith("s_cbranch_scc") and t < a and i + 1 < len(rows):
            a2, src2, ins2 = rows[i + 1]
            t2 = branch_target(a2, ins2)
            if ins2.startswith("s_branch") and t2 is not None and t2 < a2 and src2 == src:
                head = (t2, a)  # common path start, back edge
    if head is None:
        sys.exit("loop not found")
    start, end = head
    c, files = collections.Counter(), collections.Counter()
    scratch_hot = 0
    for a, src, ins in rows[by_addr[start]:by_addr[end] + 1]:
        k = cls(ins)
        c[k] += 1
        if k.startswith("valu"):
            files[src.split(":")[0]] += 1
        scratch_hot += ins.startswith("scratch_")
    print(f"# {SYM}: common frame path 0x{start:x}..0x{end:x} (one wave-frame, 8 games)")
    for k in ("valu", "valu (transcendental)", "salu", "lds", "memory"):
        print(f"  {k:24s} {c[k]}")
    print(f"  VALU total               {c['valu'] + c['valu (transcendental)']}")
    print("  VALU by source file: " + ", ".join(f"{f} {n}" for f, n in files.most_common()))
    print(f"  scratch instructions on the path: {scratch_hot}")
    sc = collections.Counter((src, ins.split()[0]) for a, src, ins in rows if ins.startswith("scratch_"))
    print(f"# scratch instructions in the kernel: {sum(sc.values())}, by source line")
    for (src, op), n in sorted(sc.items()):
        print(f"  {n:4d} {op:24s} {src}")


if __name__ == "__main__":
    main()
