"""Per-kernel register / LDS / spill record of the BUILT library, read from the gfx950 code objects'
AMDGPU metadata notes (what the loader allocates), not from a compiler remark.

    python tools/kernel_resources.py [--lib fastgaussianprocesses_amd/_lib/libfgp_hip.so] [--grep k_fwd_cols_r2c]

Copies the .so to a temporary directory, unbundles it there (llvm-objdump --offloading), and prints
for every kernel: arch VGPRs, AGPRs, SGPRs, spills, group (LDS) segment bytes, and the waves per SIMD
that the registers allow (MI355X_MICROARCH.md 'Register files': allocation granule 8, 512 per lane).
"""
import argparse
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def waves_per_simd(vgpr, agpr):
    # gfx950: unified 512-entry file; the AGPRs start at accum_offset = ceil(vgpr / 4) * 4
    total = (((vgpr + 3) // 4) * 4 + agpr) if agpr else vgpr
    alloc = ((max(total, 1) + 7) // 8) * 8
    return min(8, 512 // alloc)


def read_kernels(lib):
    tmp = tempfile.mkdtemp()
    try:
        so = os.path.join(tmp, "lib.so")
        shutil.copy(lib, so)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        out = {}
        for co in sorted(glob.glob(os.path.join(tmp, "lib.so.*gfx950*"))):
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                   stdout=subprocess.PIPE).stdout.decode(errors="replace")
            # one YAML map per kernel, keys in alphabetical order: an entry starts at its .agpr_count;
            # the kernel is named by its .symbol (argument maps carry .name keys of their own)
            cur = None
            for line in notes.splitlines():
                if re.match(r"\s*-\s+\.agpr_count:", line):
                    cur = {}
                m = re.match(r"\s*-?\s*\.(agpr_count|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|"
                             r"group_segment_fixed_size|private_segment_fixed_size|symbol):\s+(\S+)", line)
                if m and cur is not None:
                    k, v = m.group(1), m.group(2)
                    cur[k] = int(v) if v.lstrip("-").isdigit() else v
                    if k == "symbol":
                        out[v[:-3] if v.endswith(".kd") else v] = cur
        return {k: v for k, v in out.items() if "vgpr_count" in v}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def demangle(names):
    r = subprocess.run([shutil.which("c++filt") or os.path.join(LLVM, "llvm-cxxfilt")], input="\n".join(names).encode(), stdout=subprocess.PIPE)
    return r.stdout.decode().splitlines()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=os.path.join(ROOT, "fastgaussianprocesses_amd", "_lib", "libfgp_hip.so"))
    p.add_argument("--grep", default="")
    a = p.parse_args()
    ks = read_kernels(a.lib)
    names = sorted(ks)
    dem = demangle(names)
    print("%-70s %5s %5s %5s %6s %6s %7s %5s" % ("kernel", "vgpr", "agpr", "sgpr", "vspill", "sspill", "lds", "w/simd"))
    for mangled, nice in zip(names, dem):
        if a.grep and not re.search(a.grep, nice):
            continue
        k = ks[mangled]
        short = nice.split("(")[0].replace("void ", "")
        print("%-70s %5d %5d %5d %6d %6d %7d %5d" % (short[:70], k.get("vgpr_count", 0), k.get("agpr_count", 0),
                                                   k.get("sgpr_count", 0), k.get("vgpr_spill_count", 0),
                                                   k.get("sgpr_spill_count", 0), k.get("group_segment_fixed_size", 0),
                                                   waves_per_simd(k.get("vgpr_count", 0), k.get("agpr_count", 0))))


if __name__ == "__main__":
    sys.exit(main())
