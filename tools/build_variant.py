"""Build an experiment variant of libpong_ga.so into ab/NAME.so: the
product build's sources and flags (pong_amd/build.py) plus extra defines,
objects in ab/NAME.obj/ so the product objects stay untouched.  ab/ is
git-ignored but travels with gpurun (an A/B needs the variant on the box);
delete it when the A/B is done.

    python tools/build_variant.py NAME [-DPG_TIMELINE ...]
    PONG_GA_LIB=ab/NAME.so python tools/sweep.py ...
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "neuro-genetic-pong-self-play_amd"))
from pong_amd import build as B  # noqa: E402


def main(argv):
    name, extra = argv[0], argv[1:]
    out_dir = os.path.join(REPO, "ab")
    obj_dir = os.path.join(out_dir, name + ".obj")
    os.makedirs(obj_dir, exist_ok=True)
    flags = [f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC",
             "-Wall", "-Wno-unused-function", "-I", os.path.join(B.REPO_DIR, "include")] + extra
    procs, objs = [], []
    for uname, src, uflags in B.UNITS:
        src = os.path.join(B.CSRC, src)
        obj = os.path.join(obj_dir, uname + ".o")
        cmd = [B.HIPCC] + flags + B.SOURCE_FLAGS.get(os.path.basename(src), []) + uflags + ["-c", "-o", obj, src]
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    lib = os.path.join(out_dir, name + ".so")
    subprocess.check_call([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-o", lib] + objs)
    print(lib)


if __name__ == "__main__":
    main(sys.argv[1:])
