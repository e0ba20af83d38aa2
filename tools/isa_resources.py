"""Per-kernel ISA resources of the built library (VGPR/AGPR/SGPR counts,
spills, private segment bytes per lane, scratch instructions): the line
profiles/<round>/isa_resources.txt publishes.

The library's .hip_fatbin section holds one offload bundle per translation
unit; each bundle's gfx950 code object is read with llvm-readelf --notes
(the kernel descriptors' metadata) and llvm-objdump -d (scratch_* memory
instructions per kernel).

    python tools/isa_resources.py [lib.so] [--all] > profiles/r03/isa_resources.txt
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "gfx950"
# kernels on the evaluation path (the rest are listed with --all)
HOT = ("k_service<8, 16, 3", "k_prep_records<8, 16, 3", "k_wide<", "k_decide<4, 16, 3", "k_fitness", "k_merge",
       "k_hof", "k_scatter", "k_order", "k_inherit", "k_iota", "k_cand_keys", "k_vary", "k_select", "k_schedule",
       "k_row_hash", "k_forward_general")


def code_objects(lib):
    """The gfx950 code objects of every offload bundle in lib's .hip_fatbin."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fb}", lib, os.path.join(td, "x")],
                       check=True, capture_output=True)
        data = open(fb, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        q = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if TARGET in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, pos + 1)
    return out


def kernels(co_bytes):
    """[(name, fields)] from the code object's metadata notes, plus scratch instruction counts."""
    with tempfile.NamedTemporaryFile(suffix=".elf") as fh:
        fh.write(co_bytes)
        fh.flush()
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", fh.name], check=True, capture_output=True,
                               text=True).stdout
        dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", fh.name], check=True,
                             capture_output=True, text=True).stdout
    scratch, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            scratch[cur] = 0
        elif cur and re.search(r"\sscratch_(load|store)", line):
            scratch[cur] += 1
    out, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"^\s*-?\s*\.(\w+):\s+(.*)$", line)
        if not m:
            continue
        key, val = m.group(1), m.group(2).strip()
        if key == "agpr_count" and line.lstrip().startswith("-"):
            cur = {"agpr_count": val}
            out.append(cur)
        elif cur is not None and key in ("name", "vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                                         "private_segment_fixed_size", "group_segment_fixed_size", "wavefront_size"):
            cur[key] = val
    res = []
    for k in out:
        name = k.get("name", "?")
        k["scratch_insts"] = str(scratch.get(name, 0))
        res.append((name, k))
    return res


def demangle(names):
    p = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return p.stdout.splitlines() if p.returncode == 0 else names


def main(argv):
    lib = next((a for a in argv if not a.startswith("--")),
               os.path.join(REPO, "neuro-genetic-pong-self-play_amd", "libpong_ga.so"))
    show_all = "--all" in argv
    rows = {}
    for co in code_objects(lib):
        for name, k in kernels(co):
            rows[name] = k
    names = sorted(rows)
    pretty = dict(zip(names, demangle(names)))
    print(f"# {os.path.basename(lib)}: gfx950 kernel resources (llvm-readelf --notes; scratch_* from llvm-objdump)")
    print(f"{'kernel':64s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'vspill':>6s} {'sspill':>6s} "
          f"{'priv_B':>6s} {'lds_B':>6s} {'scratch_insts':>13s}")
    for name in names:
        pn = re.sub(r"^void ", "", pretty[name].replace("(anonymous namespace)::", "").split("(")[0]).replace("pg::", "")
        if not show_all and not pn.startswith(HOT):
            continue
        k = rows[name]
        print(f"{pn[:64]:64s} {k.get('vgpr_count', '?'):>5s} {k.get('agpr_count', '?'):>5s} "
              f"{k.get('sgpr_count', '?'):>5s} {k.get('vgpr_spill_count', '?'):>6s} {k.get('sgpr_spill_count', '?'):>6s} "
              f"{k.get('private_segment_fixed_size', '?'):>6s} {k.get('group_segment_fixed_size', '?'):>6s} "
              f"{k['scratch_insts']:>13s}")


if __name__ == "__main__":
    main(sys.argv[1:])
