"""Disassembly of one kernel of the built library (gfx950), for instruction
counts of a kernel's hot path:

    python tools/isa_dump.py [lib.so] SYMBOL_SUBSTRING > out.s
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_resources as R  # noqa: E402


def main(argv):
    lib = argv[0] if len(argv) > 1 else os.path.join(R.REPO, "neuro-genetic-pong-self-play_amd", "libpong_ga.so")
    sym = argv[-1]
    for co in R.code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".elf") as fh:
            fh.write(co)
            fh.flush()
            dis = subprocess.run([f"{R.LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", fh.name], check=True,
                                 capture_output=True, text=True).stdout
        on = False
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                on = sym in m.group(1)
                if on:
                    base = int(line.split()[0], 16)
                    print(line)
                continue
            if on and line.strip():
                # "insn operands  // ADDR: ENCODING <sym+0xOFF>" -> "OFF: insn operands [-> target]"
                m = re.match(r"^\s*(.*?)\s*// ([0-9A-F]+):[^<]*(?:<[^+>]*\+(0x[0-9a-f]+)>)?", line)
                if m:
                    tgt = f"   -> {m.group(3)}" if m.group(3) else ""
                    print(f"{int(m.group(2), 16) - base:x}: {m.group(1)}{tgt}")
                else:
                    print(line.rstrip())


if __name__ == "__main__":
    main(sys.argv[1:])
