"""Build the in-tree HIP library fastgaussianprocesses_amd/_lib/libfgp_hip.so for gfx950.

    python -m fastgaussianprocesses_amd.build [--force]

hipcc cross-compiles without a GPU.  The .so is git-ignored but travels to the GPU box with the
gpurun snapshot; it is rebuilt only when a source is newer than it (or --force).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIB_DIR, "libfgp_hip.so")
OBJ_DIR = os.path.join(LIB_DIR, "obj")
SOURCES = ["fgp_runtime.hip", "fgp_transforms.hip", "fgp_nll.hip", "fgp_nll_re.hip", "fgp_predict.hip", "fgp_multitask.hip", "fgp_points.hip",
           "fgp_spectral.hip"]
HEADERS = ["fgp_common.h", "fgp_runtime.h", "fgp_nll.h"]
# gfx950 (MI355X) only: the kernels' inter-workgroup hand-offs rely on gfx9 store counting (csrc/fgp_spectral.hip
# refuses to compile for other families)
ARCH = os.environ.get("FGP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _inputs():
    root = os.path.dirname(HERE)
    return ([os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(root, "include", "fgp_hip.h")])


def needs_build():
    if not os.path.isfile(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in _inputs())


def build(force=False, verbose=True):
    if not force and not needs_build():
        return LIB
    os.makedirs(OBJ_DIR, exist_ok=True)
    objs = []
    procs = []
    hdr_t = max(os.path.getmtime(p) for p in _inputs() if not p.endswith(".hip"))
    for src in SOURCES:
        obj = os.path.join(OBJ_DIR, src.replace(".hip", ".o"))
        objs.append(obj)
        srcp = os.path.join(CSRC, src)
        # per-source objects (git- and gpurun-ignored): a source is recompiled when it or a header changed
        if not force and os.path.isfile(obj) and os.path.getmtime(obj) > max(hdr_t, os.path.getmtime(srcp)):
            continue
        cmd = [HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=" + ARCH, "-fPIC", "-c", srcp, "-o", obj]
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError("hipcc failed: %s\n%s" % (" ".join(cmd), out.decode(errors="replace")))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stdout.decode(errors="replace")))
    os.replace(tmp, LIB)
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
