"""Instruction count of k_service's common frame path, by source phase.

Walks the line-annotated disassembly (llvm-objdump -d -l of a
-gline-tables-only device object) from the frame loop's head, skipping every
conditional branch whose skipped range is mostly RARE source lines (game
start, serve, hidden-ball jump, certificate failure paths, rally check, game
end, tracing), and counts the instructions met per phase until the loop's
back edge.  A static model: no latencies, the common case only (ball visible
in every game of the wave, no face crossing, every certificate passing).

    hipcc ... -gline-tables-only --cuda-device-only --no-gpu-bundle-output -c -o k.o pong_ga.hip
    llvm-objdump -d -l --no-show-raw-insn --disassemble-symbols=SYM k.o > k.s
    python tools/isa_hotpath.py k.s
"""
import collections
import re
import sys

# (file suffix, first line, last line, phase) -- ranges of the sources; the
# first match wins.  "rare" ranges are skipped when a branch jumps over them.
PHASES = [  # pg_service.hpp line ranges of round 3's k_service (adjust after edits)
    ("pg_service.hpp", 161, 186, "rare:start"),
    ("pg_service.hpp", 194, 203, "hidden-jump gate"),
    ("pg_service.hpp", 204, 215, "rare:hidden-jump"),
    ("pg_service.hpp", 246, 294, "rare:cert-fail"),
    ("pg_service.hpp", 308, 313, "rare:trace"),
    ("pg_service.hpp", 334, 335, "rally gate"),
    ("pg_service.hpp", 336, 358, "rare:rally"),
    ("pg_service.hpp", 360, 400, "rare:game-end"),
    ("pg_service.hpp", 216, 228, "physics+features"),
    ("pg_service.hpp", 229, 245, "network+certify"),
    ("pg_service.hpp", 295, 307, "decision-exchange+clamp"),
    ("pg_service.hpp", 314, 319, "no-score counter"),
    ("pg_service.hpp", 359, 359, "termination test"),
    ("pg_service.hpp", 150, 160, "loop"),
    ("pg_device.hpp", 144, 155, "rare:serve"),
    ("pg_device.hpp", 102, 120, "rare:face"),
    ("pg_device.hpp", 133, 143, "rare:hidden-jump"),
    ("pg_device.hpp", 56, 132, "physics+features"),
    ("pg_device.hpp", 196, 202, "physics+features"),
    ("pg_device.hpp", 204, 217, "decision-exchange+clamp"),
    ("pg_device.hpp", 225, 260, "network+certify"),
    ("pg_device.hpp", 156, 195, "rare:rally"),
    ("pg_cascade.hpp", 587, 700, "rare:cert-fail"),
    ("pg_cascade.hpp", 800, 830, "rare:cert-fail"),
    ("pg_cascade.hpp", 1, 2000, "network+certify"),
    ("__clang_hip_math.h", 1, 100000, "math (fmin/fmax/exp)"),
]


def phase_of(loc):
    if loc is None:
        return "?"
    f, ln = loc
    for suf, lo, hi, ph in PHASES:
        if f.endswith(suf) and lo <= ln <= hi:
            return ph
    return "other:" + f.rsplit("/", 1)[-1] + ":" + str(ln)


def parse(path):
    insts = []  # (addr, text, loc)
    loc = None
    for line in open(path):
        m = re.match(r"^; (/\S+):(\d+)", line)
        if m:
            loc = (m.group(1), int(m.group(2)))
            continue
        m = re.match(r"^\s+(\S.*?)\s*// ([0-9A-F]+):", line)
        if m:
            insts.append((int(m.group(2), 16), m.group(1), loc))
    return insts


def main(path):
    insts = parse(path)
    by_addr = {a: i for i, (a, _, _) in enumerate(insts)}

    def target(text, addr):
        m = re.search(r"s_c?branch\w*\s+(-?\d+)", text)
        off = int(m.group(1))
        if off >= 32768:
            off -= 65536
        return addr + 4 + 4 * off

    # the loop head: the first instruction of the game-start block's branch
    start = next(i for i, (_, _, l) in enumerate(insts) if l and phase_of(l) == "rare:start")
    # back up to the branch that skips it
    i = start
    while not insts[i][1].startswith("s_cbranch"):
        i -= 1
    counts = collections.Counter()
    kinds = collections.Counter()
    seen = 0
    while seen < 5000:
        seen += 1
        addr, text, loc = insts[i]
        op = text.split()[0]
        ph = phase_of(loc)
        if op.startswith("s_cbranch"):
            t = target(text, addr)
            j = by_addr.get(t)
            if j is None:
                break
            if j < i:  # a backward branch: the frame loop's back edge (or a rare inner loop)
                if seen > 50:
                    break
                i += 1
                continue
            skipped = [phase_of(l) for _, _, l in insts[i + 1:j]]
            rare = sum(1 for p in skipped if p.startswith("rare"))
            counts[(ph, "SALU")] += 1
            if skipped and rare * 2 >= len(skipped):
                i = j
            else:
                i += 1
            continue
        if op == "s_branch":
            t = target(text, addr)
            j = by_addr.get(t)
            counts[(ph, "SALU")] += 1
            if j is None or j < i:
                break
            i = j
            continue
        cls = ("VALU" if op.startswith("v_") else "SALU" if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_nop", "s_load", "s_buffer")) else
               "wait/nop" if op.startswith(("s_waitcnt", "s_nop")) else "SMEM" if op.startswith(("s_load", "s_buffer")) else
               "LDS" if op.startswith("ds_") else "VMEM" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "other")
        counts[(ph, cls)] += 1
        if cls == "VALU" and (op.startswith(("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq"))):
            counts[(ph, "trans")] += 1
        kinds[op] += cls == "VALU"
        i += 1
    phases = sorted({p for p, _ in counts})
    print(f"{'phase':28s} {'VALU':>5s} {'trans':>5s} {'SALU':>5s} {'wait/nop':>8s} {'LDS':>4s} {'VMEM':>4s}")
    tot = collections.Counter()
    for p in phases:
        row = [counts[(p, c)] for c in ("VALU", "trans", "SALU", "wait/nop", "LDS", "VMEM")]
        for c, v in zip(("VALU", "trans", "SALU", "wait/nop", "LDS", "VMEM"), row):
            tot[c] += v
        print(f"{p:28s} {row[0]:5d} {row[1]:5d} {row[2]:5d} {row[3]:8d} {row[4]:4d} {row[5]:4d}")
    print(f"{'total':28s} {tot['VALU']:5d} {tot['trans']:5d} {tot['SALU']:5d} {tot['wait/nop']:8d} {tot['LDS']:4d} {tot['VMEM']:4d}")
    print("most frequent VALU:", ", ".join(f"{k} {v}" for k, v in kinds.most_common(12)))


if __name__ == "__main__":
    main(sys.argv[1])
