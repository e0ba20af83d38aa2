"""Instruction count of k_service's common frame path, by source phase.

Walks the line-annotated disassembly (llvm-objdump -d -l of a
-gline-tables-only device object) from the frame loop's head, skipping every
conditional branch whose skipped range is mostly RARE source lines (game
start, serve, hidden-ball jump, certificate failure paths, rally check, game
end, tracing), and counts the instructions met per phase until the loop's
back edge.  A static model: no latencies, the common case only (ball visible
in every game of the wave, no face crossing, every certificate passing); the
walk assumes rare blocks lie between a branch and its target, so a layout that
moves them out of line (wave-uniform branches) can end it early -- compare
builds with the GPU A/B, not with this count alone.

    hipcc ... -gline-tables-only --cuda-device-only --no-gpu-bundle-output -c -o k.o pong_ga.hip
    llvm-objdump -d -l --no-show-raw-insn --disassemble-symbols=SYM k.o > k.s
    python tools/isa_hotpath.py k.s
"""
import collections
import re
import sys

# (file suffix, first line, last line, phase) -- ranges of the sources; the
# first match wins.  "rare" ranges are skipped when a branch jumps over them.
CSRC = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))), "neuro-genetic-pong-self-play_amd", "csrc")

# (file, first-line anchor, last-line anchor, phase): source ranges found by
# the text of their first and last lines (substring match, first occurrence
# at or after the previous anchor of the same file); the first range that
# contains a line wins.  "rare" ranges are skipped when a branch jumps over them.
ANCHORS = [
    ("pg_service.hpp", "if (fresh) {  // start game w", "g_fails = g_slow = 0;", "rare:start", 2),
    ("pg_service.hpp", "const bool hid =", "if (!kTrace && __builtin_amdgcn_ballot_w64", "hidden-jump gate"),
    ("pg_service.hpp", "const int h = st.timer - 1;", "hidden += h;", "rare:hidden-jump"),
    ("pg_service.hpp", "if (PG_ANY(idx < 0) && idx < 0) {  // rare", "lds_st(&slots[sx].flag, 0);", "rare:cert-fail"),
    ("pg_service.hpp", "if (p.trace) {  // a wave-uniform test first", "(vis << 4));", "rare:trace"),
    ("pg_service.hpp", "if (__builtin_expect(__builtin_amdgcn_ballot_w64(!left_nn)", "if (kind == kOppScore", "rare:scripted"),
    ("pg_service.hpp", "PG_PP(pp_rally,", "timeout >= kRallyStart && timeout <= kTimeoutThresh) {", "rally gate"),
    ("pg_service.hpp", "const int rs = (threadIdx.x / L) * 2;  // the group's side-0 slot", "slots[rs].rally_span = 2 *", "rare:rally"),
    ("pg_service.hpp", "if (lig == 0) finish_game(p, w, st, frames, total);", "fresh = true;", "rare:game-end"),
    ("pg_service.hpp", "const int s1b = st.s1, s2b = st.s2;", "int left = 0, right = 0;", "physics+features"),
    ("pg_service.hpp", "if (vis) {  // get_actions", "PG_PP(pp_fail, idx < 0);", "network+certify"),
    ("pg_service.hpp", "const int mine = index_to_code(idx);", "act_r = clamp_action(rc2, right);", "decision-exchange+clamp"),
    ("pg_service.hpp", "{  // calculate_timeout_and_frames", "rally_at = -1;  // the next rally", "no-score counter"),
    ("pg_service.hpp", "const bool over = st.s1 >= kWinScore", "if (PG_ANY(over) && over) {", "termination test"),
    ("pg_service.hpp", "while (w < games_total) {", "while (w < games_total) {", "loop"),
    ("pg_device.hpp", "__device__ void serve() {", "point += 1;", "rare:serve"),
    ("pg_device.hpp", "if (PG_ANY(face) && face) {", "vis = 0;", "rare:face"),
    ("pg_device.hpp", "if (PG_ANY(!play) && !play) {", "if (timer == 0 && !done()) serve();", "rare:hidden-countdown"),
    ("pg_device.hpp", "const int bc2 = 2 * by + kBallH - 1, pc2", "lpy = one_player ? move(", "rare:one-player"),
    ("pg_device.hpp", "__device__ static int drift(", "return py + kPaddleSpeed", "rare:hidden-jump"),
    ("pg_device.hpp", "__device__ inline uint64_t rally_key(", "return k;", "rare:rally"),
    ("pg_device.hpp", "struct Pong {", "__device__ void serve() {", "physics+features"),
    ("pg_device.hpp", "__device__ inline int paddle_c2(", "return lo + hi;", "physics+features"),
    ("pg_device.hpp", "__device__ inline int clamp_action(", "__device__ inline int index_to_code", "decision-exchange+clamp"),
    ("pg_device.hpp", "return (int)__builtin_amdgcn_ubfe(9u", "return (int)__builtin_amdgcn_ubfe(9u", "decision-exchange+clamp"),
    ("pg_device.hpp", "template <int CTRL>", "__device__ __forceinline__ float group_sum", "network+certify"),
    ("pg_device.hpp", "__device__ __forceinline__ float group_sum", "return v;", "network+certify"),
    ("pg_cascade.hpp", "__device__ __forceinline__ int plateau_f32(", "// Plateau certificate, tried first", "rare:cert-fail"),
    ("pg_cascade.hpp", "__device__ __forceinline__ uint64_t memo_key(", "}", "rare:cert-fail"),
    ("pg_cascade.hpp", "struct NetP {", "__device__ __forceinline__ int plateau_f32(", "network+certify"),
]
PHASES = []


def _resolve():
    import os
    cache = {}
    for f, a0, a1, ph, *extra in ANCHORS:
        if f not in cache:
            cache[f] = open(os.path.join(CSRC, f)).read()
        text = cache[f]
        i0 = text.find(a0)
        if i0 < 0:
            print(f"warning: anchor not found in {f}: {a0!r}", file=sys.stderr)
            continue
        i1 = text.find(a1, i0)
        if i1 < 0:
            i1 = i0
        l0 = text.count("\n", 0, i0) + 1
        l1 = text.count("\n", 0, i1 + len(a1)) + 1 + (extra[0] if extra else 0)
        PHASES.append((f, l0, l1, ph))
    PHASES.append(("__clang_hip_math.h", 1, 10 ** 6, "math (fmin/fmax/exp)"))


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
    _resolve()
    insts = parse(path)
    by_addr = {a: i for i, (a, _, _) in enumerate(insts)}

    def target(text, addr):
        m = re.search(r"s_c?branch\w*\s+(-?\d+)", text)
        off = int(m.group(1))
        if off >= 32768:
            off -= 65536
        return addr + 4 + 4 * off

    # the loop head: the first conditional branch that jumps over (mostly) the game-start block
    i = None
    for k, (addr, text, _) in enumerate(insts):
        if not text.startswith("s_cbranch"):
            continue
        j = by_addr.get(target(text, addr))
        if j is None or j <= k + 8:
            continue
        sk = [phase_of(l) for _, _, l in insts[k + 1:j]]
        if sum(p == "rare:start" for p in sk) * 2 >= len(sk):
            i = k
            break
    def rareness(x):
        n = r = 0
        while x < len(insts) and n < 40:
            t = insts[x][1]
            if t.startswith(("s_cbranch", "s_branch")):
                break
            n += 1
            r += phase_of(insts[x][2]).startswith("rare")
            x += 1
        return r / n if n else 0.0

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
